"""On-GPU data pipeline — the reference's dataset module (/root/reference/dataset.py)
for frames already decoded to uint8.

The reference reads each TIFF with ``cv2.imread``, resizes (INTER_AREA /
INTER_NEAREST), normalises (2/98 percentile clip, CLAHE 2.0 / 8x8, min-max)
and binarises the mask per image on the host, one image at a time with
``num_workers=0`` (dataset.py:30-66, 121-138); its augmenter writes augmented
copies to ``temp_augmentation/`` on disk (dataset.py:140-210).  Here the same
per-image arithmetic runs as HIP kernels (``csrc/data.hip``) over a whole batch
of frames resident in HBM, and augmented frames stay in HBM:

* ``preprocess`` — resize + normalise + mask binarisation of [N, H, W] uint8
  frames into [N, 1, h, w] float32 images / masks (``CellSegmentationDataset``
  semantics, dataset.py:44-66).
* ``CellSegmentationDataset`` / ``prepare_data`` — the reference's dataset and
  loader API over in-memory frames; batches come out already on the GPU.
* ``CellAugmenter`` — ``augment_training_data`` returns originals + augmented
  frames.  ``A.RandomRotate90`` and ``A.VerticalFlip`` (dataset.py:147,150) are
  index-exact HIP transforms; ``A.Affine`` and ``A.AdvancedBlur``
  (dataset.py:148-149,151: interpolating, p=0.3 each) are not built and are
  reported as skipped.

TIFF decoding (``cv2.imread``) and directory listing (``load_original_data``)
stay on the host: pass decoded frames (e.g. ``np.asarray(PIL.Image.open(p))``).
"""
from __future__ import annotations

import warnings
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib


def _frames(x, device) -> torch.Tensor:
    """[N, H, W] uint8 device tensor from a tensor / array / list of equal-size frames."""
    if isinstance(x, torch.Tensor):
        t = x
    elif isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x))
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.stack([np.asarray(f) for f in x])))
    if t.dtype != torch.uint8:
        raise TypeError(f"frames must be uint8 (cv2.IMREAD_GRAYSCALE), got {t.dtype}")
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() != 3:
        raise ValueError(f"frames must be [N, H, W], got {tuple(t.shape)}")
    return t.to(device).contiguous()


def preprocess(images, masks=None, img_size: Tuple[int, int] = (256, 256), normalize: bool = True,
               device=None):
    """dataset.py:44-66 for a batch: uint8 frames [N, H, W] -> float32
    images [N, 1, h, w] (INTER_AREA resize + normalize_microscopy_image) and
    masks [N, 1, h, w] (INTER_NEAREST resize, > 0).  ``img_size`` is cv2's
    (width, height)."""
    device = torch.device(device or "cuda")
    _lib.require_gpu(torch.empty(0, device=device))
    lib = _lib.load()
    st = _lib.stream_handle(device)
    ow, oh = img_size
    x = _frames(images, device)
    n, h, w = x.shape
    if oh > h or ow > w:
        # cv2.resize(INTER_AREA) falls back to an area-weighted bilinear
        # interpolation when enlarging; only the downscaling area path (the
        # reference's microscopy frames are larger than img_size) is built
        raise NotImplementedError(
            f"preprocess: frames {h}x{w} are smaller than img_size {oh}x{ow}; INTER_AREA upscaling "
            "(dataset.py:51) is not implemented on the GPU path")
    if (h, w) != (oh, ow):
        r = torch.empty((n, oh, ow), dtype=torch.uint8, device=device)
        _lib.check(lib.unet_resize_area_u8(x.data_ptr(), n, h, w, r.data_ptr(), oh, ow, st), "unet_resize_area_u8")
        x = r
    out = torch.empty((n, 1, oh, ow), dtype=torch.float32, device=device)
    _lib.check(lib.unet_normalize_microscopy(x.data_ptr(), n, oh, ow, out.data_ptr(), 1 if normalize else 0, st),
               "unet_normalize_microscopy")
    if masks is None:
        return out
    m = _frames(masks, device)
    if m.shape[0] != n:
        raise ValueError("images and masks differ in count")
    y = torch.empty((n, 1, oh, ow), dtype=torch.float32, device=device)
    _lib.check(lib.unet_mask_prep(m.data_ptr(), n, m.shape[1], m.shape[2], y.data_ptr(), oh, ow, st),
               "unet_mask_prep")
    return out, y


def rot90_vflip(frames, k: Sequence[int], vflip: Sequence[int], device=None) -> torch.Tensor:
    """Per frame ``np.rot90(f, k[i])`` then (``vflip[i]``) ``[::-1]`` on the GPU."""
    device = torch.device(device or "cuda")
    x = _frames(frames, device)
    n, h, w = x.shape
    ks = torch.as_tensor(list(k), dtype=torch.int32, device=device)
    fs = torch.as_tensor(list(vflip), dtype=torch.int32, device=device)
    if ks.numel() != n or fs.numel() != n:
        raise ValueError("one k and one vflip per frame")
    if h != w and bool((ks % 2).any()):
        raise ValueError("odd k (90/270 degree) rotations need square frames in a batch")
    out = torch.empty_like(x)
    _lib.check(_lib.load().unet_rot90_vflip_u8(x.data_ptr(), n, h, w, ks.data_ptr(), fs.data_ptr(), out.data_ptr(),
                                               _lib.stream_handle(device)), "unet_rot90_vflip_u8")
    return out


class CellSegmentationDataset:
    """dataset.py:17-66 over decoded uint8 frames (one size per dataset)."""

    def __init__(self, images, masks, img_size: Tuple[int, int] = (256, 256), normalize: bool = True,
                 device=None):
        self.device = torch.device(device or "cuda")
        self.images = _frames(images, self.device)
        self.masks = _frames(masks, self.device)
        self.img_size = img_size
        self.normalize = normalize
        self._cache = None

    def __len__(self):
        return self.images.shape[0]

    def _all(self):
        if self._cache is None:  # the whole set in one pass of the kernels
            self._cache = preprocess(self.images, self.masks, self.img_size, self.normalize, self.device)
        return self._cache

    def __getitem__(self, idx):
        x, y = self._all()
        return x[idx], y[idx]


class GpuLoader:
    """``DataLoader(dataset, batch_size, shuffle)`` (dataset.py:136-138) whose
    batches are slices of device tensors (no host copies, no workers)."""

    def __init__(self, dataset: CellSegmentationDataset, batch_size: int = 2, shuffle: bool = True, seed: int = 0):
        self.dataset, self.batch_size, self.shuffle = dataset, batch_size, shuffle
        self.gen = torch.Generator().manual_seed(seed)

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        x, y = self.dataset._all()
        n = len(self.dataset)
        order = torch.randperm(n, generator=self.gen) if self.shuffle else torch.arange(n)
        order = order.to(x.device)
        for i in range(0, n, self.batch_size):
            idx = order[i:i + self.batch_size]
            yield x[idx], y[idx]


def prepare_data(images, masks, batch_size: int = 2, img_size: Tuple[int, int] = (256, 256),
                 shuffle: bool = True, device=None) -> GpuLoader:
    """dataset.py:121-138 over decoded frames: a loader of device batches."""
    return GpuLoader(CellSegmentationDataset(images, masks, img_size, device=device), batch_size, shuffle)


class CellAugmenter:
    """dataset.py:140-210 in HBM: ``augment_training_data(images, masks)``
    returns originals + ``augmentations_per_image`` augmented copies of each
    frame (uint8 [N, H, W] tensors) instead of file paths.  Per copy, as the
    reference's pipeline order: RandomRotate90 (p=0.5, k uniform in 0..3),
    VerticalFlip (p=0.5); the interpolating Affine / AdvancedBlur steps are not
    built (reported once)."""

    def __init__(self, augmentations_per_image: int = 3, seed: Optional[int] = None, device=None):
        self.augmentations_per_image = augmentations_per_image
        self.rng = np.random.default_rng(seed)
        self.device = torch.device(device or "cuda")
        self.skipped = ("Affine", "AdvancedBlur")
        self._warned = False

    def augment_training_data(self, train_images, train_masks):
        x = _frames(train_images, self.device)
        m = _frames(train_masks, self.device)
        if self.augmentations_per_image == 0:
            return x, m
        if not self._warned:
            warnings.warn("CellAugmenter: A.Affine and A.AdvancedBlur (dataset.py:148-151) are not built on the "
                          "GPU path; RandomRotate90 and VerticalFlip are applied", RuntimeWarning)
            self._warned = True
        n = x.shape[0]
        a = self.augmentations_per_image
        reps = n * a
        rot = self.rng.random(reps) < 0.5
        k = np.where(rot, self.rng.integers(0, 4, reps), 0)
        if x.shape[1] != x.shape[2]:
            k = np.where(k % 2 == 1, (k + 1) % 4, k)  # keep non-square frames' shape: 90 -> 180, 270 -> 0
        flip = (self.rng.random(reps) < 0.5).astype(np.int64)
        src_x = x.repeat_interleave(a, dim=0)
        src_m = m.repeat_interleave(a, dim=0)
        mb = (src_m > 0).to(torch.uint8) * 255  # dataset.py:166
        ax = rot90_vflip(src_x, k.tolist(), flip.tolist(), self.device)
        am = rot90_vflip(mb, k.tolist(), flip.tolist(), self.device)
        self.last_params = {"k": k, "vflip": flip}
        return torch.cat([x, ax]), torch.cat([m, am])

    def cleanup(self):
        """Nothing on disk to remove (dataset.py:204-207 deletes temp_augmentation/)."""

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.cleanup()
        return False


def load_original_data(data_dir: str = "manual_labels", image_type: str = "W"):
    """dataset.py:69-118 lists TIFF paths and cv2.imread decodes them on the host;
    neither is on the GPU path."""
    raise NotImplementedError("file listing / TIFF decoding stay on the host: decode the frames and pass them to "
                              "CellSegmentationDataset / prepare_data")
