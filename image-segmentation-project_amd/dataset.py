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
  frames through the reference's whole pipeline (dataset.py:148-154):
  ``A.RandomRotate90`` / ``A.VerticalFlip`` (index-exact), ``A.Affine``
  (cv2.warpAffine's fixed-point bilinear / nearest) and ``A.AdvancedBlur``
  (cv2.filter2D), with the reference's probabilities.

TIFF decoding (``cv2.imread``) and directory listing (``load_original_data``)
stay on the host: pass decoded frames (e.g. ``np.asarray(PIL.Image.open(p))``).
"""
from __future__ import annotations

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
    elif len(x) and all(isinstance(f, torch.Tensor) for f in x):
        t = torch.stack([f.to(device) for f in x])
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.stack([np.asarray(f) for f in x])))
    if t.dtype != torch.uint8:
        raise TypeError(f"frames must be uint8 (cv2.IMREAD_GRAYSCALE), got {t.dtype}")
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() != 3:
        raise ValueError(f"frames must be [N, H, W], got {tuple(t.shape)}")
    return t.to(device).contiguous()


def _mixed(x) -> bool:
    """A list / tuple of frames that do not all share one shape."""
    return isinstance(x, (list, tuple)) and len({tuple(np.shape(f)) for f in x}) > 1


def preprocess(images, masks=None, img_size: Tuple[int, int] = (256, 256), normalize: bool = True,
               device=None):
    """dataset.py:44-66 for a batch: uint8 frames [N, H, W] -> float32
    images [N, 1, h, w] (INTER_AREA resize + normalize_microscopy_image) and
    masks [N, 1, h, w] (INTER_NEAREST resize, > 0).  ``img_size`` is cv2's
    (width, height)."""
    device = torch.device(device or "cuda")
    _lib.require_gpu(torch.empty(0, device=device))
    if _mixed(images):  # frames of several sizes (e.g. augmented non-square frames): one pass per size
        shapes = [tuple(np.shape(f)) for f in images]
        ow, oh = img_size
        out = torch.empty((len(images), 1, oh, ow), dtype=torch.float32, device=device)
        y = torch.empty_like(out) if masks is not None else None
        for shp in dict.fromkeys(shapes):
            idx = [i for i, t in enumerate(shapes) if t == shp]
            r = preprocess([images[i] for i in idx], None if masks is None else [masks[i] for i in idx],
                           img_size, normalize, device)
            it = torch.as_tensor(idx, device=device)
            if masks is None:
                out.index_copy_(0, it, r)
            else:
                out.index_copy_(0, it, r[0])
                y.index_copy_(0, it, r[1])
        return out if masks is None else (out, y)
    lib = _lib.load()
    st = _lib.stream_handle(device)
    ow, oh = img_size
    x = _frames(images, device)
    n, h, w = x.shape
    if (h, w) != (oh, ow):
        # INTER_AREA: the area average when shrinking both axes, OpenCV's
        # fixed-point area-mode linear resize when an axis is enlarged
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
        # frames of several sizes (augmented non-square frames) stay a list
        self.images = list(images) if _mixed(images) else _frames(images, self.device)
        self.masks = list(masks) if _mixed(masks) else _frames(masks, self.device)
        self.img_size = img_size
        self.normalize = normalize
        self._cache = None

    def __len__(self):
        return len(self.images)

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
    frame (uint8 device tensors) instead of file paths, in the reference's
    order (originals, then per original its copies).  Per copy, the reference's
    pipeline (dataset.py:148-154) with its probabilities:

    1. ``A.RandomRotate90(p=0.5)``: np.rot90 by k uniform in 0..3;
    2. ``A.Affine(scale=(0.95, 1.05), translate_percent=(-0.05, 0.05),
       rotate=(-15, 15), shear=(-5, 5), p=0.3)``: x / y scale, translation and
       shear drawn independently (keep_ratio=False), the albumentations 2.0
       matrix about the image centre, applied as cv2.warpAffine (bilinear
       image, nearest mask, constant 0 border);
    3. ``A.VerticalFlip(p=0.5)`` (folded into the warp kernel's output rows);
    4. ``A.AdvancedBlur(blur_limit=(3, 7), p=0.3)`` on the image only:
       generalized-Gaussian kernel (sigma 0.2-1.0 per axis, rotation +-90 deg,
       beta 0.5-8, noise 0.9-1.1) through cv2.filter2D.

    Parameters are drawn on the host (numpy, ``seed``) — albumentations' own
    random stream cannot be reproduced — and the transforms run as HIP kernels
    (``csrc/data.hip``), bit-exact against ``oracle/dataset_ref.py`` for the
    same parameters (``last_params``).  A 90/270 degree rotation of a
    non-square frame transposes its shape, as in the reference: the result is
    then a list of frames, which ``preprocess`` / ``prepare_data`` accept (each
    frame is resized to ``img_size`` there, as the reference's dataset does)."""

    def __init__(self, augmentations_per_image: int = 3, seed: Optional[int] = None, device=None):
        self.augmentations_per_image = augmentations_per_image
        self.rng = np.random.default_rng(seed)
        self.device = torch.device(device or "cuda")
        self.last_params = None

    def _sample(self, reps: int, h: int, w: int):
        rng = self.rng
        k = np.where(rng.random(reps) < 0.5, rng.integers(0, 4, reps), 0)
        affine = rng.random(reps) < 0.3
        aff = {"scale_x": rng.uniform(0.95, 1.05, reps), "scale_y": rng.uniform(0.95, 1.05, reps),
               "tx": rng.uniform(-0.05, 0.05, reps), "ty": rng.uniform(-0.05, 0.05, reps),
               "rotate": rng.uniform(-15.0, 15.0, reps),
               "shear_x": -rng.uniform(-5.0, 5.0, reps), "shear_y": -rng.uniform(-5.0, 5.0, reps)}
        vflip = rng.random(reps) < 0.5
        blur = rng.random(reps) < 0.3
        kernels = np.zeros((reps, 7, 7), np.float32)
        ksize = np.zeros(reps, np.int64)
        from .augment_params import advanced_blur_kernel
        for i in range(reps):
            kz = int(rng.choice([3, 5, 7]))
            sx, sy = rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0)
            ang = rng.uniform(-90.0, 90.0)
            beta = rng.uniform(0.5, 1.0) if rng.random() < 0.5 else rng.uniform(1.0, 8.0)
            noise = rng.uniform(0.9, 1.1, (kz, kz))
            if blur[i]:
                kernels[i, :kz, :kz] = advanced_blur_kernel(kz, sx, sy, ang, beta, noise)
                ksize[i] = kz
        # matrices in the frame's post-rotation shape
        minv = np.zeros((reps, 6), np.float64)
        from .augment_params import affine_matrix, invert_affine
        for i in range(reps):
            hh, ww = (w, h) if k[i] % 2 else (h, w)
            if affine[i]:
                m = affine_matrix(aff["scale_x"][i], aff["scale_y"][i], aff["tx"][i], aff["ty"][i],
                                  aff["rotate"][i], aff["shear_x"][i], aff["shear_y"][i], hh, ww)
                minv[i] = invert_affine(m)
        return {"k": k, "affine": affine.astype(np.int64), "affine_params": aff, "minv": minv,
                "vflip": vflip.astype(np.int64), "blur": blur.astype(np.int64), "ksize": ksize, "kernels": kernels}

    def augment_training_data(self, train_images, train_masks):
        x = _frames(train_images, self.device)
        m = _frames(train_masks, self.device)
        if self.augmentations_per_image == 0:
            return x, m
        n, h, w = x.shape
        a = self.augmentations_per_image
        reps = n * a
        prm = self._sample(reps, h, w)
        self.last_params = prm
        src_x = x.repeat_interleave(a, dim=0)
        src_m = (m > 0).to(torch.uint8).repeat_interleave(a, dim=0) * 255  # dataset.py:177
        lib, st, dev = _lib.load(), _lib.stream_handle(self.device), self.device
        outs_x, outs_m = [None] * reps, [None] * reps
        odd = prm["k"] % 2 == 1
        groups = [np.nonzero(~odd)[0], np.nonzero(odd)[0]] if h != w else [np.arange(reps)]
        for idx in groups:
            if idx.size == 0:
                continue
            g = len(idx)
            it = torch.as_tensor(idx, device=dev)
            ks = torch.as_tensor(prm["k"][idx], dtype=torch.int32, device=dev)
            zero = torch.zeros(g, dtype=torch.int32, device=dev)
            hh, ww = (w, h) if (h != w and prm["k"][idx[0]] % 2) else (h, w)
            rx = torch.empty((g, hh, ww), dtype=torch.uint8, device=dev)
            rm = torch.empty_like(rx)
            gx, gm = src_x.index_select(0, it).contiguous(), src_m.index_select(0, it).contiguous()
            _lib.check(lib.unet_rot90_vflip_u8(gx.data_ptr(), g, h, w, ks.data_ptr(), zero.data_ptr(), rx.data_ptr(),
                                               st), "unet_rot90_vflip_u8")
            _lib.check(lib.unet_rot90_vflip_u8(gm.data_ptr(), g, h, w, ks.data_ptr(), zero.data_ptr(), rm.data_ptr(),
                                               st), "unet_rot90_vflip_u8")
            minv = torch.as_tensor(prm["minv"][idx], dtype=torch.float64, device=dev)
            act = torch.as_tensor(prm["affine"][idx], dtype=torch.int32, device=dev)
            fl = torch.as_tensor(prm["vflip"][idx], dtype=torch.int32, device=dev)
            wx, wm = torch.empty_like(rx), torch.empty_like(rm)
            _lib.check(lib.unet_warp_affine_u8(rx.data_ptr(), g, hh, ww, minv.data_ptr(), act.data_ptr(),
                                               fl.data_ptr(), 0, wx.data_ptr(), st), "unet_warp_affine_u8")
            _lib.check(lib.unet_warp_affine_u8(rm.data_ptr(), g, hh, ww, minv.data_ptr(), act.data_ptr(),
                                               fl.data_ptr(), 1, wm.data_ptr(), st), "unet_warp_affine_u8")
            kern = torch.as_tensor(prm["kernels"][idx], dtype=torch.float32, device=dev)
            kz = torch.as_tensor(prm["ksize"][idx], dtype=torch.int32, device=dev)
            bx = torch.empty_like(wx)
            _lib.check(lib.unet_filter2d_u8(wx.data_ptr(), g, hh, ww, kern.data_ptr(), kz.data_ptr(), bx.data_ptr(),
                                            st), "unet_filter2d_u8")
            for j, i in enumerate(idx.tolist()):
                outs_x[i], outs_m[i] = bx[j], wm[j]
        if all(t.shape == (h, w) for t in outs_x):
            return torch.cat([x, torch.stack(outs_x)]), torch.cat([m, torch.stack(outs_m)])
        # non-square frames rotated by 90 / 270 degrees: a list of frames
        return list(x.unbind(0)) + outs_x, list(m.unbind(0)) + outs_m

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
