"""Pixel-wise segmentation losses on MI355X (hot-path subset of
/root/reference/losses.py).

``BCELoss`` (:31-37), ``DiceLoss`` (:13-28, one global Dice over the whole
batch, smooth=1) and ``ComboLoss`` (:161-171, alpha*BCE + (1-alpha)*Dice) run as
one fused HIP reduction (BCE terms, sum sigma*y, sum sigma, sum y in fp64) plus
a fused gradient kernel.  ``get_loss_function`` (:345-403) keeps the registry
behaviour: default 'combo', unknown names print a warning and fall back to
ComboLoss.  The other twelve reference losses are outside the hot path
 and raise ``NotImplementedError``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib

BCE, DICE, COMBO = 0, 1, 2


class _FusedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, kind, alpha, smooth):
        _lib.require_gpu(logits, target)
        lib = _lib.load()
        x = logits.contiguous().float()
        t = target.to(device=x.device, dtype=torch.float32).contiguous()
        if x.numel() != t.numel():
            raise ValueError(f"logits {tuple(x.shape)} and target {tuple(t.shape)} differ in size")
        sums, scratch = _lib.loss_buffers(x.device)
        out = torch.empty((), dtype=torch.float32, device=x.device)
        _lib.check(lib.unet_loss_forward(x.data_ptr(), t.data_ptr(), x.numel(), kind, float(alpha), float(smooth),
                                         sums.data_ptr(), scratch.data_ptr(), scratch.numel(), out.data_ptr(),
                                         _lib.stream_handle(x.device)),
                   "unet_loss_forward")
        ctx.save_for_backward(x, t, sums)
        ctx.cfg = (kind, float(alpha), float(smooth))
        ctx.in_shape = logits.shape
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, t, sums = ctx.saved_tensors
        kind, alpha, smooth = ctx.cfg
        g = grad_out.contiguous().float()
        dl = torch.empty_like(x)
        _lib.check(_lib.load().unet_loss_backward(x.data_ptr(), t.data_ptr(), x.numel(), kind, alpha, smooth,
                                                  sums.data_ptr(), g.data_ptr(), dl.data_ptr(),
                                                  _lib.stream_handle(x.device)), "unet_loss_backward")
        return dl.view(ctx.in_shape), None, None, None, None


class DiceLoss(nn.Module):
    """losses.py:13-28 — 1 - (2*sum(sigma*y) + smooth) / (sum sigma + sum y + smooth)."""

    def __init__(self, smooth=1.0):
        super().__init__()
        self.smooth = smooth

    def forward(self, pred, target):
        return _FusedLoss.apply(pred, target, DICE, 0.0, self.smooth)


class BCELoss(nn.Module):
    """losses.py:31-37 — F.binary_cross_entropy_with_logits, mean reduction."""

    def forward(self, pred, target):
        return _FusedLoss.apply(pred, target, BCE, 1.0, 1.0)


class ComboLoss(nn.Module):
    """losses.py:161-171 — alpha * BCE + (1 - alpha) * Dice."""

    def __init__(self, alpha=0.5, smooth=1.0):
        super().__init__()
        self.alpha = alpha
        self.smooth = smooth

    def forward(self, pred, target):
        return _FusedLoss.apply(pred, target, COMBO, self.alpha, self.smooth)


_NOT_ON_PATH = ("weighted_bce", "balanced_bce", "focal", "triple_combo", "tversky", "tversky_balanced",
                "tversky_recall", "focal_tversky", "sensitivity_specificity", "log_cosh_dice",
                "exponential_logarithmic", "distance_map_bce", "hausdorff", "boundary")


def get_loss_function(config):
    """losses.py:345-403: build the criterion named by ``config['loss_fn']``."""
    name = config.get("loss_fn", "combo")
    if name == "dice":
        return DiceLoss(smooth=config.get("smooth", 1.0))
    if name == "bce":
        return BCELoss()
    if name == "combo":
        return ComboLoss(alpha=config.get("loss_alpha", 0.5))
    if name in _NOT_ON_PATH:
        raise NotImplementedError(f"loss '{name}' is outside the MI355X hot path (SURVEY.md §2 row 2)")
    print(f"Warning: Unknown loss function '{name}', defaulting to ComboLoss")
    return ComboLoss(alpha=config.get("loss_alpha", 0.5))
