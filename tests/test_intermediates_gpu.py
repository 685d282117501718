"""Layer-by-layer parity of every forward activation and activation gradient in
the native workspace against the oracle — localises any divergence to one op.

Two references:
* the fp32 oracle (the reference path itself): deviations grow with depth
  because a randomly initialised BN ResNet amplifies perturbations (the bf16
  rounding of activations); forward tolerance 0.15 on relative L2 error;
* the same oracle with bf16 rounding emulated where the HIP path stores bf16
  (printed for diagnosis: it diverges from the HIP path almost as much, which
  is what shows the deviation is amplification, not an op error — op-level
  parity is asserted at 2e-2 by test_wiring_gpu.py).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle

pytestmark = pytest.mark.gpu


class _Q(torch.autograd.Function):
    """Round to bf16 in the forward AND round the incoming gradient to bf16."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def trace_oracle(m, x, emulate=False):
    """Forward of oracle.ReferenceUNet with every intermediate kept (non-inplace)."""
    t = {}
    q = _Q.apply if emulate else (lambda v: v)

    def keep(name, v):
        v = q(v)
        v.retain_grad()
        t[name] = v
        return v

    def conv(mod, v, **kw):
        w = mod.weight.to(torch.bfloat16).float() if emulate else mod.weight
        if isinstance(mod, torch.nn.ConvTranspose2d):
            return F.conv_transpose2d(v, w, mod.bias, stride=2)
        return F.conv2d(v, w, mod.bias, stride=mod.stride, padding=mod.padding)

    def bn(mod, v):
        return F.batch_norm(v, mod.running_mean, mod.running_var, mod.weight, mod.bias, True, mod.momentum, mod.eps)

    y0 = keep("y0", conv(m.input_conv, q(x)))
    x1 = keep("x1", F.relu(bn(m.bn1, y0)))
    p0 = keep("p0", m.maxpool(x1))
    cur = p0
    for s, stage in enumerate((m.enc1, m.enc2, m.enc3, m.enc4)):
        for b, blk in enumerate(stage):
            pre = f"enc{s + 1}.{b}."
            y1 = keep(pre + "y1", conv(blk.conv1, cur))
            h = keep(pre + "h", F.relu(bn(blk.bn1, y1)))
            y2 = keep(pre + "y2", conv(blk.conv2, h))
            if blk.downsample is not None:
                yds = keep(pre + "yds", conv(blk.downsample[0], cur))
                skip = bn(blk.downsample[1], yds)
            else:
                skip = cur
            cur = keep(pre + "out", F.relu(bn(blk.bn2, y2) + skip))
            t[f"_enc{s + 1}"] = cur
    skips = {4: t["_enc3"], 3: t["_enc2"], 2: t["_enc1"], 1: x1}
    d = cur
    for lvl in (4, 3, 2, 1):
        up = getattr(m, f"upconv{lvl}")
        dec = getattr(m, f"decoder{lvl}")
        pre = f"dec{lvl}."
        u = keep(pre + "up", conv(up, d))
        cat = torch.cat((skips[lvl], u), 1)
        cat.retain_grad()
        t[pre + "cat"] = cat
        y1 = keep(pre + "y1", conv(dec[0], cat))
        h = keep(pre + "h", F.relu(bn(dec[1], y1)))
        y2 = keep(pre + "y2", conv(dec[3], h))
        d = keep(pre + "out", F.relu(bn(dec[4], y2)))
    logits = m.conv_final(m.upconv0(d))
    return logits, t


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _compare(views, tr):
    rows = []
    for name, v in views.items():
        is_grad = name.startswith("d.") or ".d." in name
        key = name.replace("d.", "") if is_grad else name
        if key not in tr:
            continue
        r = tr[key].grad if is_grad else tr[key].detach()
        if r is None:
            continue
        rows.append((name, _rel(v.cpu(), r)))
    return rows


def test_every_intermediate(pkg, golden, cuda):
    base = golden("base64.npz")
    x = torch.from_numpy(base["x"])
    y = torch.from_numpy(base["masks"])
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=0)
    results = {}
    for emulate in (False, True):
        ref.load_state_dict(sd)
        ref.train()
        logits, tr = trace_oracle(ref, x, emulate)
        oracle.bce_with_logits(logits, y).backward()
        results[emulate] = tr
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=False)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x.cuda())
    pkg.get_loss_function({"loss_fn": "bce"})(out, y.cuda()).backward()
    torch.cuda.synchronize()
    plan = m._last_plan
    # decoder1's act is not stored by a training forward (the head applies that
    # BN + ReLU to dec1.y2 itself, HeadArgs.bn_fold); its effect is in the logits
    views = {k: t for k, t in plan.tensor_views().items() if k != "dec1.out"}
    fp32 = dict(_compare(views, results[False]))
    emu = dict(_compare(views, results[True]))
    for name in emu:
        print(f"{name:22s} vs-fp32 {fp32[name]:.3e}   vs-bf16-emulated {emu[name]:.3e}")
    assert len(emu) > 100
    # forward activations: growth with depth only (no jump at any op)
    fwd = {n: e for n, e in fp32.items() if ".d." not in n and not n.startswith("d.")}
    bad = [(n, e) for n, e in fwd.items() if not e <= 0.15]
    assert not bad, bad[:20]
    # gradients: amplified at init (see test_model_gpu header); op-level parity
    # is asserted by test_wiring_gpu.py — here only require them to be finite.
    grd = {n: e for n, e in fp32.items() if n not in fwd}
    assert all(np.isfinite(e) for e in grd.values())
