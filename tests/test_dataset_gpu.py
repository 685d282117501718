"""The on-GPU data pipeline (csrc/data.hip) against the
numpy oracle (oracle/dataset_ref.py) — the reference's dataset.py:30-66 and
CellAugmenter's rot90 / vflip (dataset.py:147,150).

Bar: bit-exact.  Resized / CLAHE'd frames are uint8, masks {0, 1}, and the
normalised float32 image is computed from identical uint8 values by the same
float64 expression, so every output must be equal (torch.equal).  The cv2
parts of the oracle are parity-unpinned restatements (no OpenCV here); the
percentile part is pinned to numpy (tests/test_dataset_oracle.py).
"""
import importlib

import numpy as np
import pytest
import torch

from oracle import dataset_ref as D

pytestmark = pytest.mark.gpu


def _frames(seed, n, h, w, kind="cells"):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, size=(n, h, w), dtype=np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    out = np.empty((n, h, w), np.uint8)
    for i in range(n):
        img = rng.normal(60, 12, size=(h, w))
        for _ in range(rng.integers(5, 30)):
            cy, cx, s = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(3, 14)
            img += rng.uniform(60, 160) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        out[i] = np.clip(img, 0, 255).astype(np.uint8)
    return out


@pytest.mark.parametrize("shape,out", [((4, 512, 512), (128, 128)),   # integer factor 4
                                       ((3, 256, 256), (128, 128)),   # factor 2 (SIMD rounding)
                                       ((2, 500, 375), (128, 96)),    # fractional factors
                                       ((2, 333, 417), (128, 128))])
def test_resize_area_bit_exact(pkg, cuda, shape, out):
    lib = importlib.import_module("image-segmentation-project_amd._lib").load()
    f = _frames(0, *shape, kind="noise")
    src = torch.from_numpy(f).cuda()
    oh, ow = out
    dst = torch.empty((shape[0], oh, ow), dtype=torch.uint8, device="cuda")
    rc = lib.unet_resize_area_u8(src.data_ptr(), shape[0], shape[1], shape[2], dst.data_ptr(), oh, ow,
                                 torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    got = dst.cpu().numpy()
    for i in range(shape[0]):
        want = D.resize_area_u8(f[i], oh, ow)
        assert np.array_equal(got[i], want), (i, int((got[i] != want).sum()))


@pytest.mark.parametrize("hw", [(128, 128), (96, 160), (100, 100), (256, 250), (250, 256)])
def test_normalize_bit_exact(pkg, cuda, hw):
    f = np.concatenate([_frames(1, 3, *hw), _frames(2, 1, *hw, kind="noise"),
                        np.full((1, *hw), 77, np.uint8)])
    got = pkg.preprocess(f, img_size=(hw[1], hw[0])).cpu().numpy()
    for i in range(f.shape[0]):
        want = D.normalize_microscopy_image(f[i]).astype(np.float32)
        assert np.array_equal(got[i, 0], want), (i, float(np.abs(got[i, 0] - want).max()))
    raw = pkg.preprocess(f, img_size=(hw[1], hw[0]), normalize=False).cpu().numpy()
    assert np.array_equal(raw[:, 0], f.astype(np.float32) / np.float32(255.0))


def test_preprocess_upscale_fails_early(pkg, cuda):
    """frames smaller than img_size (cv2 INTER_AREA enlarging) are
    rejected with a clear error before any kernel runs."""
    f = np.zeros((1, 64, 64), np.uint8)
    with pytest.raises(NotImplementedError, match="upscaling"):
        pkg.preprocess(f, img_size=(128, 128))


def test_preprocess_end_to_end_matches_dataset_getitem(pkg, cuda):
    imgs = _frames(3, 4, 400, 300)
    masks = (np.random.default_rng(4).random((4, 400, 300)) < 0.3).astype(np.uint8) * 255
    x, y = pkg.preprocess(imgs, masks, img_size=(128, 128))
    assert x.shape == (4, 1, 128, 128) and y.shape == (4, 1, 128, 128)
    for i in range(4):
        wx, wy = D.preprocess(imgs[i], masks[i], img_size=(128, 128))
        assert np.array_equal(x[i].cpu().numpy(), wx), i
        assert np.array_equal(y[i].cpu().numpy(), wy), i
    # the dataset / loader API yields the same device tensors
    ds = pkg.CellSegmentationDataset(imgs, masks, img_size=(128, 128))
    a, b = ds[2]
    assert torch.equal(a, x[2]) and torch.equal(b, y[2])
    loader = pkg.prepare_data(imgs, masks, batch_size=3, img_size=(128, 128), shuffle=False)
    batches = list(loader)
    assert [t[0].shape[0] for t in batches] == [3, 1] and batches[0][0].is_cuda
    assert torch.equal(torch.cat([t[0] for t in batches]), x)


def test_augmenter_rot90_vflip_exact(pkg, cuda):
    f = _frames(5, 3, 64, 64, kind="noise")
    m = (f > 128).astype(np.uint8)
    aug = pkg.CellAugmenter(augmentations_per_image=4, seed=7)
    with pytest.warns(RuntimeWarning):
        xs, ms = aug.augment_training_data(f, m)
    assert xs.shape == (3 + 12, 64, 64) and ms.shape == xs.shape
    assert torch.equal(xs[:3].cpu(), torch.from_numpy(f))
    k, fl = aug.last_params["k"], aug.last_params["vflip"]
    for j in range(12):
        src = j // 4
        assert np.array_equal(xs[3 + j].cpu().numpy(), D.rot90_vflip(f[src], int(k[j]), bool(fl[j])))
        assert np.array_equal(ms[3 + j].cpu().numpy(), D.rot90_vflip((m[src] > 0).astype(np.uint8) * 255,
                                                                    int(k[j]), bool(fl[j])))


def test_train_model_on_frames(pkg, cuda):
    """train.py:141-157: uint8 frames go through augmentation + the GPU
    pipeline inside train_model (reference control flow)."""
    imgs = _frames(8, 6, 128, 128)
    masks = (imgs > 120).astype(np.uint8) * 255
    torch.manual_seed(0)
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=False).cuda()
    crit = pkg.get_loss_function({"loss_fn": "bce"})
    opt = pkg.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    cfg = {"batch_size": 4, "img_size": 64, "verbose": False}
    with pytest.warns(RuntimeWarning):
        res = pkg.train_model(m, imgs[:4], masks[:4], imgs[4:], masks[4:], crit, opt, None, 2,
                              torch.device("cuda"), cfg, augmentations_per_image=1)
    assert len(res["train_metrics"]) == 2 and np.isfinite(res["final_train_metrics"]["loss"])
