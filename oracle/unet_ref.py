"""TEST INFRASTRUCTURE ONLY — fp32 torch-CPU restatement of the reference hot path.

Never imported by the product package.  Every function cites the reference
file:line (under ``/root/reference``) whose behaviour it restates:

* ``ReferenceUNet`` — ``advanced_models.py:64-130,157-183,197-205,264-357``
  (``UNetWithBackbone(backbone='resnet34'|'resnet50', use_attention=False|True)``;
  ``AttentionGate`` :7-40, ``ChannelAttention`` :43-61) with the
  torchvision ResNet34 encoder (``advanced_models.py:73,81-87``; torchvision's
  ``BasicBlock`` layout: conv1/bn1/conv2/bn2/downsample.{0,1}).
* ``bce_with_logits``/``dice_loss``/``combo_loss``/``get_loss_function`` —
  ``losses.py:13-37,161-171,345-403``.
* ``calculate_metrics`` — ``utils.py:120-151``.
* ``train_step``/``train_epoch``/``evaluate`` — ``train.py:17-112``.
* ``make_adam`` — ``train.py:331-335`` (Adam, coupled L2 weight decay).

The state_dict keys and shapes are identical to the reference model, so the
same closed-form weights load into the reference, this oracle and the HIP
build.
"""
from __future__ import annotations

import math
from collections import OrderedDict, defaultdict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------
# closed-form deterministic weights (no 24 M-parameter dumps in fixtures)
# ----------------------------------------------------------------------------
def hash_uniform(stream: int, count: int) -> np.ndarray:
    """Uniform [-1, 1) float64 values from a splitmix64 hash of (stream, i)."""
    i = np.arange(count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = i + np.uint64((stream * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    top = (z >> np.uint64(40)).astype(np.float64)  # 24 random bits
    return top / float(1 << 23) - 1.0


def closed_form_state_dict(model: nn.Module, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Deterministic weights for every entry of ``model.state_dict()``.

    Conv / ConvTranspose weights: He-uniform bound sqrt(6/fan_in); biases
    1/sqrt(fan_in); BN gamma 1+0.1u, beta 0.1u, running_mean 0.05u,
    running_var 1+0.25|u|; num_batches_tracked 0.
    """
    out = OrderedDict()
    sd = model.state_dict()
    for idx, (name, t) in enumerate(sd.items()):
        stream = seed * 1000003 + idx + 1
        if name.endswith("num_batches_tracked"):
            out[name] = torch.zeros_like(t)
            continue
        u = torch.from_numpy(hash_uniform(stream, t.numel())).reshape(t.shape)
        leaf = name.rsplit(".", 1)[-1]
        owner = model.get_submodule(name.rsplit(".", 1)[0])
        if isinstance(owner, nn.BatchNorm2d):
            if leaf == "weight":
                v = 1.0 + 0.1 * u
            elif leaf == "bias":
                v = 0.1 * u
            elif leaf == "running_mean":
                v = 0.05 * u
            else:
                v = 1.0 + 0.25 * u.abs()
        else:
            w = owner.weight
            if isinstance(owner, nn.ConvTranspose2d):
                fan_in = w.shape[0]          # contraction length of the k2s2 GEMM
            else:
                fan_in = w.shape[1] * w.shape[2] * w.shape[3]
            if leaf == "weight":
                v = u * math.sqrt(6.0 / fan_in)
            else:
                v = u / math.sqrt(fan_in)
        out[name] = v.to(t.dtype).contiguous()
    return out


# ----------------------------------------------------------------------------
# model restatement
# ----------------------------------------------------------------------------
class BasicBlock(nn.Module):
    """torchvision ResNet BasicBlock (encoder of advanced_models.py:84-87)."""

    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(
                nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        h = self.relu(self.bn1(self.conv1(x)))
        h = self.bn2(self.conv2(h))
        skip = x if self.downsample is None else self.downsample(x)
        return self.relu(h + skip)


class Bottleneck(nn.Module):
    """torchvision ResNet Bottleneck, v1.5 (stride on the 3x3): the resnet50
    encoder of advanced_models.py:102-117."""

    def __init__(self, cin: int, planes: int, stride: int):
        super().__init__()
        cout = planes * 4
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        h = self.relu(self.bn1(self.conv1(x)))
        h = self.relu(self.bn2(self.conv2(h)))
        h = self.bn3(self.conv3(h))
        skip = x if self.downsample is None else self.downsample(x)
        return self.relu(h + skip)


def _stage50(cin: int, planes: int, blocks: int, stride: int) -> nn.Sequential:
    return nn.Sequential(Bottleneck(cin, planes, stride), *[Bottleneck(planes * 4, planes, 1) for _ in range(blocks - 1)])


def _stage(cin: int, cout: int, blocks: int, stride: int) -> nn.Sequential:
    layers = [BasicBlock(cin, cout, stride)]
    layers += [BasicBlock(cout, cout, 1) for _ in range(blocks - 1)]
    return nn.Sequential(*layers)


def decoder_block(cin: int, cout: int) -> nn.Sequential:
    """advanced_models.py:197-205: [Conv3x3(bias) -> BN -> ReLU] x 2."""
    return nn.Sequential(
        nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
        nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class AttentionGate(nn.Module):
    """advanced_models.py:7-40: psi = sigmoid(BN(conv1x1(relu(BN(W_g g) + BN(W_x x))))); x * psi."""

    def __init__(self, f_g: int, f_l: int, f_int: int):
        super().__init__()
        self.W_g = nn.Sequential(nn.Conv2d(f_g, f_int, 1, 1, 0, bias=True), nn.BatchNorm2d(f_int))
        self.W_x = nn.Sequential(nn.Conv2d(f_l, f_int, 1, 1, 0, bias=True), nn.BatchNorm2d(f_int))
        self.psi = nn.Sequential(nn.Conv2d(f_int, 1, 1, 1, 0, bias=True), nn.BatchNorm2d(1), nn.Sigmoid())
        self.relu = nn.ReLU(inplace=True)

    def forward(self, g, x):
        return x * self.psi(self.relu(self.W_g(g) + self.W_x(x)))   # :28-40


class ChannelAttention(nn.Module):
    """advanced_models.py:43-61 (squeeze-and-excitation with avg + max pooling, ratio 16)."""

    def __init__(self, c: int, reduction_ratio: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.fc = nn.Sequential(nn.Conv2d(c, c // reduction_ratio, 1, bias=False), nn.ReLU(inplace=True),
                                nn.Conv2d(c // reduction_ratio, c, 1, bias=False))
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        return x * self.sigmoid(self.fc(self.avg_pool(x)) + self.fc(self.max_pool(x)))   # :56-61


class ReferenceUNet(nn.Module):
    """UNetWithBackbone(n_classes, 'resnet34', pretrained=False, use_attention).

    Registration order (hence state_dict order) follows advanced_models.py:76-100,
    157-160.  ``width`` multiplies every channel count (1 = reference; 2 =
    the build-defined "wide" config of SURVEY.md §0).
    """

    def __init__(self, n_classes: int = 1, width: int = 1, use_attention: bool = False, backbone: str = "resnet34"):
        super().__init__()
        self.use_attention = use_attention
        c0 = 64 * width
        self.input_conv = nn.Conv2d(1, c0, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(c0)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        if backbone == "resnet50":   # advanced_models.py:102-130 (torchvision resnet50 layers)
            c = [256, 512, 1024, 2048]
            self.enc1 = _stage50(64, 64, 3, 1)
            self.enc2 = _stage50(256, 128, 4, 2)
            self.enc3 = _stage50(512, 256, 6, 2)
            self.enc4 = _stage50(1024, 512, 3, 2)
            up1 = d1 = 64
            att = [(1024, 1024, 512), (512, 512, 256), (256, 256, 128), (64, 64, 32)]   # :175-183
        else:                        # advanced_models.py:72-100
            c = [c0, 2 * c0, 4 * c0, 8 * c0]
            self.enc1 = _stage(c[0], c[0], 3, 1)
            self.enc2 = _stage(c[0], c[1], 4, 2)
            self.enc3 = _stage(c[1], c[2], 6, 2)
            self.enc4 = _stage(c[2], c[3], 3, 2)
            up1 = d1 = c0 // 2
            att = [(c[2], c[2], c[1]), (c[1], c[1], c[0]), (c[0], c[0], c0 // 2), (c0 // 2, c0, c0 // 2)]
        self.upconv4 = nn.ConvTranspose2d(c[3], c[2], 2, 2)
        self.decoder4 = decoder_block(2 * c[2], c[2])
        self.upconv3 = nn.ConvTranspose2d(c[2], c[1], 2, 2)
        self.decoder3 = decoder_block(2 * c[1], c[1])
        self.upconv2 = nn.ConvTranspose2d(c[1], c[0], 2, 2)
        self.decoder2 = decoder_block(2 * c[0], c[0])
        self.upconv1 = nn.ConvTranspose2d(c[0], up1, 2, 2)
        self.decoder1 = decoder_block(c0 + up1, d1)
        self.upconv0 = nn.ConvTranspose2d(d1, c0 // 4, 2, 2)          # :158-159
        self.conv_final = nn.Conv2d(c0 // 4, n_classes, 1)
        if use_attention:   # advanced_models.py:163-183, registered after conv_final
            for lvl, (fg, fl, fi) in zip((4, 3, 2, 1), att):
                setattr(self, f"attention{lvl}", AttentionGate(fg, fl, fi))
            for lvl, ch in zip((4, 3, 2, 1), (c[2], c[1], c[0], d1)):
                setattr(self, f"ch_attention{lvl}", ChannelAttention(ch))

    def _level(self, lvl: int, skip, up):
        """One decoder level: skip-first concat (+ attention gate / channel attention, :286-334)."""
        dec = getattr(self, f"decoder{lvl}")
        if not self.use_attention:
            return dec(torch.cat((skip, up), 1))
        skip = getattr(self, f"attention{lvl}")(g=up, x=skip)
        return getattr(self, f"ch_attention{lvl}")(dec(torch.cat((skip, up), 1)))

    def forward(self, x):
        x1 = self.relu(self.bn1(self.input_conv(x)))          # :268-270
        x2 = self.enc1(self.maxpool(x1))                      # :272-273
        x3 = self.enc2(x2)
        x4 = self.enc3(x3)
        x5 = self.enc4(x4)                                    # :276
        d = self._level(4, x4, self.upconv4(x5))             # :284-293
        d = self._level(3, x3, self.upconv3(d))              # :295-303
        d = self._level(2, x2, self.upconv2(d))              # :305-313
        u = self.upconv1(d)                                   # :315
        if u.shape != x1.shape:                               # :318-325 crop
            dh, dw = x1.shape[2] - u.shape[2], x1.shape[3] - u.shape[3]
            if dh > 0 and dw > 0:
                x1 = x1[:, :, dh // 2:dh // 2 + u.shape[2], dw // 2:dw // 2 + u.shape[3]]
        d = self._level(1, x1, u)                             # :327-334
        d0 = self.upconv0(d)                                  # :337
        if d0.shape[2] != x.shape[2] or d0.shape[3] != x.shape[3]:   # :340-347
            dh, dw = d0.shape[2] - x.shape[2], d0.shape[3] - x.shape[3]
            if dh > 0 or dw > 0:
                d0 = d0[:, :, dh // 2:dh // 2 + x.shape[2], dw // 2:dw // 2 + x.shape[3]]
        return self.conv_final(d0)                            # :350


class TinyUNet(nn.Module):
    """BASELINE config 1 (no reference equivalent): one down/up
    level with 8 channels, built only from the reference's block vocabulary:
    ``_decoder_block`` (advanced_models.py:197-205), maxpool 3/2/1 (:83),
    ``ConvTranspose2d(k2,s2)`` (:90), skip-first concat (:292), 1x1 head (:160).
    """

    def __init__(self, n_classes: int = 1, ch: int = 8):
        super().__init__()
        self.enc = decoder_block(1, ch)
        self.pool = nn.MaxPool2d(3, 2, 1)
        self.mid = decoder_block(ch, 2 * ch)
        self.up = nn.ConvTranspose2d(2 * ch, ch, 2, 2)
        self.dec = decoder_block(2 * ch, ch)
        self.conv_final = nn.Conv2d(ch, n_classes, 1)

    def forward(self, x):
        e = self.enc(x)
        m = self.mid(self.pool(e))
        return self.conv_final(self.dec(torch.cat((e, self.up(m)), 1)))


# ----------------------------------------------------------------------------
# losses (losses.py) and metrics (utils.py)
# ----------------------------------------------------------------------------
def bce_with_logits(logits, target):
    """losses.py:31-37 — mean over every element."""
    return F.binary_cross_entropy_with_logits(logits, target)


def dice_loss(logits, target, smooth: float = 1.0):
    """losses.py:13-28 — ONE global Dice over the whole batch."""
    p = torch.sigmoid(logits).reshape(-1)
    t = target.reshape(-1)
    inter = (p * t).sum()
    return 1 - (2.0 * inter + smooth) / (p.sum() + t.sum() + smooth)


def combo_loss(logits, target, alpha: float = 0.5, smooth: float = 1.0):
    """losses.py:161-171."""
    return alpha * bce_with_logits(logits, target) + (1 - alpha) * dice_loss(logits, target, smooth)


class _Loss(nn.Module):
    def __init__(self, fn, **kw):
        super().__init__()
        self.fn, self.kw = fn, kw

    def forward(self, logits, target):
        return self.fn(logits, target, **self.kw)


def get_loss_function(config: dict) -> nn.Module:
    """losses.py:345-403 restricted to the hot-path names; unknown -> combo."""
    name = config.get("loss_fn", "combo")
    if name == "bce":
        return _Loss(bce_with_logits)
    if name == "dice":
        return _Loss(dice_loss, smooth=config.get("smooth", 1.0))
    return _Loss(combo_loss, alpha=config.get("loss_alpha", 0.5))


def calculate_metrics(pred, target) -> dict:
    """utils.py:120-151 — fp32 sums over the whole batch, eps 1e-7."""
    pb = (pred > 0.5).float().reshape(-1)
    t = target.reshape(-1)
    tp = (pb * t).sum().item()
    fp = (pb * (1 - t)).sum().item()
    fn = ((1 - pb) * t).sum().item()
    tn = ((1 - pb) * (1 - t)).sum().item()
    eps = 1e-7
    precision = tp / (tp + fp + eps)
    recall = tp / (tp + fn + eps)
    return {
        "precision": precision,
        "recall": recall,
        "f1": 2 * precision * recall / (precision + recall + eps),
        "iou": tp / (tp + fp + fn + eps),
        "accuracy": (tp + tn) / (tp + tn + fp + fn + eps),
    }


# ----------------------------------------------------------------------------
# train loop (train.py)
# ----------------------------------------------------------------------------
def make_adam(model, lr: float = 1e-3, weight_decay: float = 1e-5):
    """train.py:331-335 — torch Adam with coupled L2 weight decay."""
    return torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)


def train_step(model, optimizer, criterion, images, masks):
    """One iteration of train.py:38-60; returns (logits, loss, batch_metrics)."""
    logits = model(images)
    loss = criterion(logits, masks)
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    with torch.no_grad():
        m = calculate_metrics(torch.sigmoid(logits), masks)
    return logits, loss, m


def train_epoch(model, loader, optimizer, criterion, device) -> dict:
    """train.py:17-68 — batch-size-weighted means of per-batch metrics."""
    model.train()
    acc = defaultdict(float)
    n = 0
    total = 0.0
    for images, masks in loader:
        images, masks = images.to(device), masks.to(device)
        _, loss, m = train_step(model, optimizer, criterion, images, masks)
        b = images.size(0)
        for k, v in m.items():
            acc[k] += v * b
        n += b
        total += loss.item() * b
    for k in acc:
        acc[k] /= n
    acc["loss"] = total / n
    return acc


def evaluate(model, loader, device, criterion) -> dict:
    """train.py:71-112."""
    model.eval()
    acc = defaultdict(float)
    n = 0
    with torch.no_grad():
        for images, masks in loader:
            images, masks = images.to(device), masks.to(device)
            logits = model(images)
            loss = criterion(logits, masks)
            m = calculate_metrics(torch.sigmoid(logits), masks)
            b = images.size(0)
            for k, v in m.items():
                acc[k] += v * b
            acc["loss"] += loss.item() * b
            n += b
    for k in acc:
        acc[k] /= n
    return acc
