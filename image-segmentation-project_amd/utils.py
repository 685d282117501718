"""Metrics and helpers of the training loop (/root/reference/utils.py:120-190).

``calculate_metrics`` keeps the reference aggregation exactly: foreground
counts pooled over the whole batch from ``pred > 0.5``, then precision /
recall / f1 / iou / accuracy with eps 1e-7 in Python floats (so an empty
prediction on an empty mask gives IoU 0, utils.py:142).  The counts come from
one HIP reduction (exact fp64 sums) and ONE device->host copy instead of the
reference's four ``.item()`` syncs.
"""
from __future__ import annotations

import torch

from . import _lib

EPS = 1e-7


def metrics_from_counts(tp: float, fp: float, fn: float, tn: float) -> dict:
    """utils.py:135-151 formula on already-reduced counts."""
    precision = tp / (tp + fp + EPS)
    recall = tp / (tp + fn + EPS)
    f1 = 2 * precision * recall / (precision + recall + EPS)
    iou = tp / (tp + fp + fn + EPS)
    accuracy = (tp + tn) / (tp + tn + fp + fn + EPS)
    return {"precision": precision, "recall": recall, "f1": f1, "iou": iou, "accuracy": accuracy}


def mask_counts(values, target, from_logits: bool):
    """Device fp64 tensor [8]; [4:8] = tp, fp, fn, tn (no host sync)."""
    _lib.require_gpu(values, target)
    v = values.contiguous().float()
    t = target.to(device=v.device, dtype=torch.float32).contiguous()
    sums, scratch = _lib.loss_buffers(v.device)
    _lib.check(_lib.load().unet_mask_metrics(v.data_ptr(), t.data_ptr(), v.numel(), 0 if from_logits else 1,
                                             sums.data_ptr(), scratch.data_ptr(), scratch.numel(),
                                             _lib.stream_handle(v.device)), "unet_mask_metrics")
    return sums


def calculate_metrics(pred, target) -> dict:
    """utils.py:120-151: ``pred`` are probabilities (sigmoid outputs)."""
    c = mask_counts(pred, target, from_logits=False)[4:8].tolist()
    return metrics_from_counts(*c)


def calculate_metrics_from_logits(logits, target) -> dict:
    """Same as ``calculate_metrics(torch.sigmoid(logits), target)`` with the mask
    decided bit-exactly as the reference's fp32 CPU sigmoid does."""
    c = mask_counts(logits, target, from_logits=True)[4:8].tolist()
    return metrics_from_counts(*c)


def get_device():
    """utils.py:153-167 — the ROCm GPU when present (torch's 'cuda' device)."""
    if torch.cuda.is_available():
        print("Using CUDA device")
        return torch.device("cuda")
    print("Using CPU")
    return torch.device("cpu")


class EarlyStopping:
    """utils.py:174-190 — stop after ``patience`` non-improving steps."""

    def __init__(self, patience=10, min_delta=0.001):
        self.patience = patience
        self.min_delta = min_delta
        self.counter = 0
        self.best_score = None
        self.early_stop = False

    def step(self, current_score):
        improved = self.best_score is None or current_score > self.best_score + self.min_delta
        if improved:
            self.best_score = current_score
            self.counter = 0
        else:
            self.counter += 1
            self.early_stop = self.early_stop or self.counter >= self.patience
        return self.early_stop
