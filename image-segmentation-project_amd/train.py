"""Training loop on MI355X — the API of /root/reference/train.py:17-364.

``train_epoch`` / ``evaluate`` keep the reference's per-batch semantics
(forward, criterion, ``zero_grad`` after the forward, backward, ``step``; train
metrics from the pre-step logits in train-mode BN; batch-size-weighted means of
per-batch metrics, train.py:38-68,89-112).  What changes is where the work
runs: the model/criterion are the HIP path, the per-batch mask counts are one
fused kernel on the logits, and the five ``.item()`` syncs per batch become one
device->host copy per epoch.

``train_model`` keeps the epoch loop control of train.py:115-244 (ReduceLROnPlateau
on val IoU, best-state deepcopy, EarlyStopping, returned dict) but takes
in-memory tensors instead of image paths: the cv2/albumentations data pipeline
is outside the hot path.
"""
from __future__ import annotations

import copy
import time
from collections import defaultdict
from typing import Dict, Optional

import torch

from .utils import EarlyStopping, mask_counts, metrics_from_counts


def _batch_record(logits, masks, loss, n):
    counts = mask_counts(logits.detach(), masks, from_logits=True)[4:8]
    return counts, loss.detach().reshape(1).float(), n


def _finish(records, with_loss_key: bool) -> Dict:
    if not records:
        return defaultdict(float)
    counts = torch.stack([r[0] for r in records]).cpu().tolist()
    losses = torch.cat([r[1] for r in records]).cpu().tolist()
    out = defaultdict(float)
    total = 0
    loss_sum = 0.0
    for (c, loss_v, (_, _, b)) in zip(counts, losses, records):
        m = metrics_from_counts(*c)
        for k, v in m.items():
            out[k] += v * b
        loss_sum += loss_v * b  # == loss.item() (fp32 value as Python float)
        total += b
    for k in list(out):
        out[k] /= total
    if with_loss_key:
        out["loss"] = loss_sum / total
    return out


def train_epoch(model: torch.nn.Module, loader, optimizer: torch.optim.Optimizer, criterion: torch.nn.Module,
                device: torch.device) -> Dict:
    """train.py:17-68."""
    model.train()
    records = []
    for images, masks in loader:
        images = images.to(device, non_blocking=True)
        masks = masks.to(device, non_blocking=True)
        outputs = model(images)
        loss = criterion(outputs, masks)
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
        with torch.no_grad():
            records.append(_batch_record(outputs, masks, loss, images.size(0)))
    return _finish(records, with_loss_key=True)


def evaluate(model: torch.nn.Module, loader, device: torch.device, criterion: torch.nn.Module) -> Dict:
    """train.py:71-112 (eval-mode BN, no grad)."""
    model.eval()
    records = []
    with torch.no_grad():
        for images, masks in loader:
            images = images.to(device, non_blocking=True)
            masks = masks.to(device, non_blocking=True)
            outputs = model(images)
            loss = criterion(outputs, masks)
            records.append(_batch_record(outputs, masks, loss, images.size(0)))
    return _finish(records, with_loss_key=True)


class GraphedTrainStep:
    """One training step (forward, criterion, zero_grad, backward, optimizer.step)
    captured into a single HIP graph and replayed: removes the per-launch host
    cost of the ~250 kernels of a step.  Inputs are static device tensors; pass
    new batches through ``__call__`` (copied in before replay).  The optimizer
    must be capturable (``optim.Adam``, or ``torch.optim.Adam(..., capturable=True)``).
    Drop every reference to an earlier eager step's loss/outputs before building
    one: a live autograd graph keeps AccumulateGrad nodes bound to the stream
    they were created on, and HIP stream capture aborts on them."""

    def __init__(self, model, criterion, optimizer, images, masks, warmup: int = 3):
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.x = images.clone()
        self.y = masks.clone()
        # the backward seed dL/dL = 1, made once in the warmup: loss.backward()
        # would fill a fresh ones tensor inside every replay (one more kernel)
        self._seed = None
        # the captured kernels write this plan's workspace, events and side
        # stream: keep it alive (and un-evictable) for the graph's lifetime
        self._plan = model._plan_for(self.x)
        self._plan.pins += 1
        for g in optimizer.param_groups:
            if not g.get("capturable", False):
                raise ValueError("GraphedTrainStep needs an optimizer built with capturable=True")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._step()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            out, loss = self._step()
        # replay rewrites these buffers in place; detached, they do not keep the
        # captured step's autograd graph alive
        self.out, self.loss = out.detach(), loss.detach()

    def _step(self):
        out = self.model(self.x)
        loss = self.criterion(out, self.y)
        self.optimizer.zero_grad(set_to_none=True)
        if self._seed is None or self._seed.shape != loss.shape or self._seed.dtype != loss.dtype:
            self._seed = torch.ones_like(loss)
        loss.backward(self._seed)
        self.optimizer.step()
        return out, loss

    def __del__(self):
        plan = getattr(self, "_plan", None)
        if plan is not None:
            plan.pins -= 1

    def __call__(self, images=None, masks=None):
        if images is not None:
            self.x.copy_(images, non_blocking=True)
            self.y.copy_(masks, non_blocking=True)
        self.graph.replay()
        return self.out, self.loss


def _is_frames(x) -> bool:
    """uint8 [N,H,W] frames (tensor, array or list of 2-D arrays)?"""
    if isinstance(x, torch.Tensor):
        return x.dtype == torch.uint8
    import numpy as np
    if isinstance(x, np.ndarray):
        return x.dtype == np.uint8
    return isinstance(x, (list, tuple)) and len(x) > 0 and getattr(x[0], "dtype", None) in (np.uint8, torch.uint8)


class TensorLoader:
    """Minimal in-memory replacement for ``prepare_data`` (dataset.py:121-138)."""

    def __init__(self, images, masks, batch_size, shuffle=False, seed=0):
        self.images = torch.as_tensor(images)
        self.masks = torch.as_tensor(masks)
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.gen = torch.Generator().manual_seed(seed)

    def __len__(self):
        return (len(self.images) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.images)
        order = torch.randperm(n, generator=self.gen) if self.shuffle else torch.arange(n)
        for i in range(0, n, self.batch_size):
            idx = order[i:i + self.batch_size]
            yield self.images[idx], self.masks[idx]


def train_model(model, train_images, train_masks, val_images, val_masks, criterion, optimizer,
                scheduler: Optional[object], num_epochs: int, device, config: Dict,
                augmentations_per_image: int = 0, save_plots: bool = True) -> Dict:
    """train.py:115-244 epoch loop.  Inputs are either preprocessed float
    tensors [N,1,H,W] or decoded uint8 frames [N,H,W] (``cv2.imread`` output);
    frames go through the on-GPU data pipeline (dataset.py: augmentation,
    resize to ``config['img_size']``, normalisation) exactly where the
    reference calls CellAugmenter / prepare_data (train.py:141-157)."""
    if isinstance(train_images, (list, tuple)) and train_images and isinstance(train_images[0], str):
        raise NotImplementedError("file paths need host TIFF decoding (cv2.imread): pass decoded uint8 frames")
    if _is_frames(train_images):
        from .dataset import CellAugmenter, prepare_data
        size = config.get("img_size", (256, 256))
        size = (size, size) if isinstance(size, int) else tuple(size)
        if augmentations_per_image > 0:
            train_images, train_masks = CellAugmenter(augmentations_per_image).augment_training_data(
                train_images, train_masks)
        train_loader = prepare_data(train_images, train_masks, config["batch_size"], size, shuffle=True,
                                    device=device)
        val_loader = prepare_data(val_images, val_masks, config["batch_size"], size, shuffle=False, device=device)
    else:
        if augmentations_per_image:
            raise ValueError("augmentation works on uint8 frames (before resize / normalisation), as the "
                             "reference's CellAugmenter does; pass frames, not preprocessed tensors")
        train_loader = TensorLoader(train_images, train_masks, config["batch_size"], shuffle=True)
        val_loader = TensorLoader(val_images, val_masks, config["batch_size"], shuffle=False)
    train_hist, val_hist, lr_hist = [], [], []
    best_iou, best_state, best_epoch = 0.0, None, 0
    stopper = EarlyStopping(patience=config.get("early_stopping_patience", 7),
                            min_delta=config.get("early_stopping_min_delta", 0.001))
    verbose = config.get("verbose", True)
    start = time.time()
    train_metrics = val_metrics = None
    for epoch in range(num_epochs):
        train_metrics = train_epoch(model, train_loader, optimizer, criterion, device)
        train_hist.append(train_metrics)
        val_metrics = evaluate(model, val_loader, device, criterion)
        val_hist.append(val_metrics)
        if scheduler is not None:
            if isinstance(scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                scheduler.step(val_metrics["iou"])
            else:
                scheduler.step()
        lr = optimizer.param_groups[0]["lr"]
        lr_hist.append(lr)
        if verbose:
            print(f"Epoch {epoch + 1:3d}/{num_epochs} - Train Loss: {train_metrics['loss']:.4f}, "
                  f"Train IoU: {train_metrics['iou']:.4f}, Val Loss: {val_metrics['loss']:.4f}, "
                  f"Val IoU: {val_metrics['iou']:.4f}, LR: {lr:.6f}")
        if val_metrics["iou"] > best_iou:
            best_iou = val_metrics["iou"]
            best_state = copy.deepcopy(model.state_dict())
            best_epoch = epoch
        if stopper.step(val_metrics["iou"]):
            if verbose:
                print(f"Early stopping triggered at epoch {epoch + 1}")
            break
    elapsed = time.time() - start
    if best_state is not None:
        model.load_state_dict(best_state)
    return {"train_metrics": train_hist, "val_metrics": val_hist, "lr_history": lr_hist, "best_iou": best_iou,
            "best_epoch": best_epoch, "best_model_state": best_state, "training_time": elapsed,
            "final_train_metrics": train_metrics, "final_val_metrics": val_metrics}


def quick_train(model, train_images, train_masks, val_images, val_masks, config: Dict, device=None,
                augmentations_per_image: int = 0) -> Dict:
    """train.py:301-364: Adam (coupled L2; the fused HIP Adam of optim.py) + ReduceLROnPlateau(max, 0.5, thr 0.01, min 1e-6)."""
    from .losses import get_loss_function
    from .optim import Adam
    from .utils import get_device
    device = device or get_device()
    model = model.to(device)
    criterion = get_loss_function(config)
    optimizer = Adam(model.parameters(), lr=config.get("learning_rate", 1e-3),
                     weight_decay=config.get("weight_decay", 1e-5))
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="max", factor=0.5,
                                                           patience=config.get("scheduler_patience", 3),
                                                           threshold=0.01, min_lr=1e-6)
    return train_model(model, train_images, train_masks, val_images, val_masks, criterion, optimizer, scheduler,
                       config.get("num_epochs", 50), device, config, augmentations_per_image,
                       config.get("save_plots", True))
