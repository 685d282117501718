"""CPU checks of the data-pipeline oracle (oracle/dataset_ref.py), SURVEY.md §8(f) row 3.

* The percentile restatement the GPU kernel follows equals numpy's own
  np.percentile (the reference's call, dataset.py:33) exactly.
* cv2 / albumentations are absent, so the resize and CLAHE
  restatements are PARITY UNPINNED; they are held to the properties the
  published algorithms guarantee: INTER_AREA at an integer factor is the
  rounded block mean; CLAHE of a constant image is one value everywhere and
  its tile LUTs are monotone; the whole normalisation maps into [0, 1] with 0
  and 1 attained; rot90 / vflip equal numpy's.
"""
import numpy as np
import pytest

from oracle import dataset_ref as D


@pytest.mark.parametrize("seed", range(6))
def test_percentile_restatement_equals_numpy(seed):
    rng = np.random.default_rng(seed)
    shape = [(17, 23), (128, 128), (64, 96), (1, 5), (300, 7), (2, 2)][seed]
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    if seed == 3:
        img[:] = 7
    for q in (0, 2, 25, 50, 97.5, 98, 100):
        assert D.percentile_linear(img, q) == float(np.percentile(img, q)), (shape, q)


def test_area_integer_factor_is_rounded_block_mean():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=(96, 128), dtype=np.uint8)
    out = D.resize_area_u8(img, 24, 32)  # factor 4
    mean = img.astype(np.float64).reshape(24, 4, 32, 4).mean(axis=(1, 3))
    assert np.abs(out.astype(np.float64) - mean).max() <= 0.5
    half = D.resize_area_u8(img, 48, 64)  # factor 2: (sum + 2) >> 2
    s = img.astype(np.int64).reshape(48, 2, 64, 2).sum(axis=(1, 3))
    assert np.array_equal(half, ((s + 2) >> 2).astype(np.uint8))


def test_area_fractional_factor_preserves_constant_and_mean():
    img = np.full((100, 75), 173, np.uint8)
    assert np.all(D.resize_area_u8(img, 64, 32) == 173)
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, size=(100, 75), dtype=np.uint8)
    out = D.resize_area_u8(img, 64, 32)
    assert abs(out.astype(np.float64).mean() - img.mean()) < 1.0


def test_clahe_properties():
    assert np.unique(D.clahe_u8(np.full((64, 64), 90, np.uint8))).size == 1
    rng = np.random.default_rng(3)
    img = rng.integers(20, 200, size=(128, 128), dtype=np.uint8)
    c = D.clahe_u8(img)
    # monotone per pixel position: a brighter input never maps darker at the same location
    c2 = D.clahe_u8(np.minimum(img.astype(np.int64) + 1, 255).astype(np.uint8))
    assert (c2.astype(np.int64) >= c.astype(np.int64) - 1).all()
    n = D.normalize_microscopy_image(img)
    assert n.dtype == np.float64 and n.min() == 0.0 and abs(n.max() - 1.0) < 1e-7


def test_clahe_padding_rule():
    """OpenCV pads both sides when either is off the grid."""
    assert D.clahe_padding(64, 64) == (0, 0)
    assert D.clahe_padding(64, 60) == (8, 4)
    assert D.clahe_padding(60, 64) == (4, 8)
    assert D.clahe_padding(100, 100) == (4, 4)


def test_rot90_vflip_matches_numpy():
    img = np.arange(48, dtype=np.uint8).reshape(6, 8)
    for k in range(4):
        assert np.array_equal(D.rot90_vflip(img, k, False), np.rot90(img, k))
        assert np.array_equal(D.rot90_vflip(img, k, True), np.rot90(img, k)[::-1])
