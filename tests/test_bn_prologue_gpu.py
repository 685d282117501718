"""BN1 + ReLU applied inside the next weight-stationary conv's halo staging
(ConvFwdArgs::xform) against the separate bn_apply pass it
replaces: the stored activations h, every later forward tensor, the logits and
the BN running statistics must be BIT-identical (the prologue evaluates
bn_apply's expression with bn_apply's coefficients), the gradients equal to
bf16 resolution (relative L2 <= 1e-2, see below), at a size where enc1 /
decoder2 / decoder1 run on the weight-stationary kernel."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(pkg, sd, x, y):
    m = pkg.UNetWithBackbone(pretrained=False)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x)
    pkg.get_loss_function({"loss_fn": "bce"})(out, y).backward()
    torch.cuda.synchronize()
    views = m._last_plan.tensor_views()
    grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    bufs = {k: b.detach().clone() for k, b in m.named_buffers()}
    return out.detach().clone(), views, grads, bufs


def test_bn_prologue_bit_identical(pkg, cuda, monkeypatch):
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in pkg.UNetWithBackbone(pretrained=False).state_dict().items()}
    xs, ms = pkg.synthetic_cells(2, 128, 128, seed=21)
    x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
    monkeypatch.delenv("UNET_NO_BN_XFORM", raising=False)
    fused = _run(pkg, sd, x, y)
    fused2 = _run(pkg, sd, x, y)
    monkeypatch.setenv("UNET_NO_BN_XFORM", "1")  # read when the native plan is created
    plain = _run(pkg, sd, x, y)
    plain2 = _run(pkg, sd, x, y)
    assert torch.equal(fused[0], plain[0])
    for k in ["enc1.0.h", "enc1.1.h", "enc1.2.h", "dec2.h", "dec1.h"]:
        assert torch.equal(fused[1][k], plain[1][k]), k
    for k, v in plain[3].items():
        assert torch.equal(fused[3][k], v), k
    # each path on its own is bit-reproducible (fixed-order weight-gradient
    # reductions; BN / loss sums are fp64 accumulations of fp32 partials)
    for a, b in ((fused, fused2), (plain, plain2)):
        diff = [k for k, v in a[2].items() if not torch.equal(v, b[2][k])]
        assert not diff, diff
    # across the two paths the backward reads bit-identical tensors, so every
    # BN-backward sum is the same set of fp32 block partials; they enter fp64
    # replica accumulators by atomic adds whose arrival order differs between
    # the two kernel sequences.  Where such an fp64 sum is not exact (partials
    # more than 2^29 apart in magnitude) its last bit follows that order, and a
    # one-ulp change of an fp32 BN coefficient (measured: 4 of 131072 elements of
    # enc1.2's dY2, 1.9e-9) flips bf16 roundings of the dZ upstream, so the two
    # paths agree to bf16 resolution (measured <= 2.5e-3 relative L2, the stem
    # weight), not bit for bit
    worst = 0.0
    for k, v in plain[2].items():
        g = fused[2][k]
        rel = ((g.double() - v.double()).norm() / v.double().norm().clamp_min(1e-30)).item()
        worst = max(worst, rel)
        assert rel <= 1e-2, (k, rel)
    print("fused vs plain gradients: worst relative L2", worst)
