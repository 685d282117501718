"""The stem by recompute (csrc/stem_rc.hip, the default for stem rows of up
to 256 pixels) against the stored-y0 stem path (UNET_STEM_RC=0: stem_fwd +
bn_relu_maxpool_fwd + maxpool_bwd + BN-fused stem_wgrad) on the same inputs
and weights (resnet34 stem, advanced_models.py:76-83).

The two paths compute y with the same MFMA sequence, but since round 6 the
recompute path normalises the fp32 y (as the reference's fp32 BatchNorm does)
while the stored path can only normalise the bf16 y0 it stored; the recompute
path also forms the stem weight gradient through the BN-backward identity
dW = k1 (dZ^T im - m1 sum im - m2 xhat^T im) instead of rounding
dY = k1 (dZ - m1 - m2 xhat) to bf16 first.  So the two differ by one bf16
rounding of y before the BN: each is pinned against ITS reference in
test_stem_production_path_vs_fp32 (recompute: the pure fp32 chain; stored:
the chain with y0 rounded to bf16), and here they are only checked to agree
within that rounding's own effect.  The recompute path's backward is
bit-reproducible.  The teacher-forced rows of test_wiring_gpu.py
(UNET_STEM_KEEP=1) pin the recompute path's dZ, bn1 and input_conv gradients
against fp32 recomputations at 2e-2.
"""
import os

import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _run(pkg, sd, x, y, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = pkg.UNetWithBackbone(pretrained=False, use_attention=False)
        m.load_state_dict(sd)
        m = m.cuda().train()
        out = m(x)
        pkg.get_loss_function({"loss_fn": "bce"})(out, y).backward()
        torch.cuda.synchronize()
        v = {k: t.detach().cpu().clone() for k, t in m._last_plan.tensor_views().items()}
        g = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
        return out.detach().cpu(), v, g
    finally:
        for k, val in old.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val


@pytest.mark.parametrize("shape", [(2, 128, 128), (4, 512, 512), (1, 64, 96)], ids=["2x128", "4x512", "1x64x96"])
def test_stem_recompute_matches_stored_path(pkg, cuda, shape):
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=3)
    xs, ms = pkg.synthetic_cells(*shape, seed=11)
    x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
    o_rc, v_rc, g_rc = _run(pkg, sd, x, y, {"UNET_STEM_RC": "1", "UNET_STEM_KEEP": "1"})
    o_st, v_st, g_st = _run(pkg, sd, x, y, {"UNET_STEM_RC": "0"})
    for k in ("x1", "p0"):
        e, same = _rel(v_rc[k], v_st[k]), (v_rc[k] == v_st[k]).float().mean().item()
        print(f"{k}: rel {e:.2e}, bit-equal fraction {same:.5f}")
        assert e <= X1_TOL_FP32, (k, e, same)
    print("logits rel", _rel(o_rc, o_st))
    assert _rel(o_rc, o_st) <= 0.10  # end-to-end bar of test_model_gpu (depth amplifies the y rounding)
    worst = sorted(((_rel(g_rc[k], g_st[k]), k) for k in g_st if g_st[k].norm() > 0), reverse=True)[:6]
    print("largest gradient differences:", [(k, f"{e:.2e}") for e, k in worst])
    # (no gradient bar here: the two paths' activations differ by a bf16
    # rounding of y, which the 30-layer random-init BN network amplifies
    # chaotically into its small cancelling BN-bias gradients -- measured up to
    # ~1.0 relative on some of them; each path's stem gradients are pinned
    # against its own reference in test_stem_production_path_vs_fp32)
    # bit-reproducible: the same step again on the recompute path
    o2, v2, g2 = _run(pkg, sd, x, y, {"UNET_STEM_RC": "1"})
    assert torch.equal(o2, o_rc)
    for k in g_rc:
        assert torch.equal(g2[k], g_rc[k]), k


def _bn_train(v, g, b, stats_from=None):
    s = v if stats_from is None else stats_from
    mean = s.mean((0, 2, 3), keepdim=True)
    var = s.var((0, 2, 3), unbiased=False, keepdim=True)
    return (v - mean) / torch.sqrt(var + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def _dskip(v):
    """the decoder1 concat gradient's skip slice (the stem output x1's second consumer)"""
    if "dec1.d.cat" in v:
        return v["dec1.d.cat"][:, :v["x1"].shape[1]]
    return v["dec1.d.cat.skip"][:, :v["x1"].shape[1]]


# measured on MI355X (profiles/r05/s2/stem_tests.txt), 2 x 256^2 | 1 x 64 x 96:
#   bf16-y0 reference: x1 1.7e-3 | 1.7e-3, p0 1.7e-3 | 1.6e-3, input_conv.weight
#     1.0e-2 | 1.4e-2, bn1.weight 1.1e-3 | 2.1e-3, bn1.bias 2.4e-3 | 3.1e-3
#   pure fp32 reference: x1 4.8e-3 | 3.8e-3, p0 3.8e-3 | 3.2e-3,
#     input_conv.weight 3.8e-2 | 6.8e-2, bn1.bias 2.4e-2 | 4.3e-2 (the weight and
#     bias gradients are small residuals of the BN backward's cancelling terms)
#   fp64 recomputation from the stored dZ: input_conv.weight 5.8e-4
X1_TOL, W_TOL = 3e-3, 3e-2   # each path against its own reference (<= 3e-2)
X1_TOL_FP32 = 8e-3            # recompute vs stored path: one bf16 rounding of y apart
W64_TOL = 2e-3


@pytest.mark.parametrize("path", ["recompute", "stored"])
@pytest.mark.parametrize("shape", [(2, 256, 256), (1, 64, 96)], ids=["2x256", "1x64x96"])
def test_stem_production_path_vs_fp32(pkg, cuda, shape, path):
    """The production stem (recompute, nothing but x1 / p0 stored) against a
    torch restatement of advanced_models.py:76,81-83 on the same bf16 input and
    weights: forward x1 = relu(bn(conv(xq))) and p0 = maxpool(x1); backward:
    the stem parameter gradients by autograd through that chain, fed the
    executor's own upstream gradients (d.p0 into the pool, the decoder1
    concat's skip slice into x1).  The recompute path normalises the fp32 conv
    output, so its reference is the pure fp32 chain of the reference model; the
    stored-y0 path (UNET_STEM_RC=0: HiRes rows wider than 256) stores y0 in
    bf16, so its reference rounds y0 to bf16 before the BN.  Both at the same
    bars: x1 / p0 <= 3e-3, every stem gradient <= 3e-2."""
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=5)
    xs, ms = pkg.synthetic_cells(*shape, seed=13)
    x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
    assert os.environ.get("UNET_STEM_KEEP") is None and os.environ.get("UNET_STEM_RC") is None
    _, v, g = _run(pkg, sd, x, y, {} if path == "recompute" else {"UNET_STEM_RC": "0"})
    if path == "recompute":
        assert "y0" not in v, "production stem path expected (no stored y0)"
    xq = x.cpu().to(torch.bfloat16).float()
    for rnd, xtol, wtol in ((path == "stored", X1_TOL, W_TOL),):
        w = sd["input_conv.weight"].to(torch.bfloat16).float().requires_grad_(True)
        gam = sd["bn1.weight"].float().clone().requires_grad_(True)
        bet = sd["bn1.bias"].float().clone().requires_grad_(True)
        y0 = torch.nn.functional.conv2d(xq, w, stride=2, padding=3)
        yq = y0
        if rnd:  # the batch statistics from the fp32 y (the statistics pass), the
            # normalisation applied to the bf16-rounded y (straight-through gradient)
            yq = y0 + (y0.detach().to(torch.bfloat16).float() - y0.detach())
        x1 = torch.relu(_bn_train(yq, gam, bet, stats_from=y0))
        p0 = torch.nn.functional.max_pool2d(x1, 3, 2, 1)
        ex1, ep0 = _rel(v["x1"], x1.detach()), _rel(v["p0"], p0.detach())
        # the pooled gradient is routed by the executor's own argmax: its x1 is
        # bf16, so windows whose fp32 maxima differ by less than a bf16 ulp tie
        # there (first index wins) and may pick another pixel than the fp32
        # reference -- a legitimate consequence of bf16 activations that
        # reroutes whole gradient values; routing both by the same argmax leaves
        # the arithmetic of the stem's backward under test
        x1v = v["x1"].float().requires_grad_(True)
        (dx1,) = torch.autograd.grad(torch.nn.functional.max_pool2d(x1v, 3, 2, 1), [x1v], [v["d.p0"].float()])
        gw, gg, gb = torch.autograd.grad([x1], [w, gam, bet], [dx1 + _dskip(v).float()])
        rows = [("input_conv.weight", _rel(g["input_conv.weight"], gw)), ("bn1.weight", _rel(g["bn1.weight"], gg)),
                ("bn1.bias", _rel(g["bn1.bias"], gb))]
        print(f"{path} path vs {'bf16-y0' if rnd else 'fp32'} reference: x1 rel {ex1:.2e}  p0 rel {ep0:.2e}  " +
              "  ".join(f"{k} {e:.2e}" for k, e in rows))
        assert ex1 <= xtol and ep0 <= xtol, (rnd, ex1, ep0)
        for k, e in rows:
            assert e <= wtol, (rnd, k, e)


def test_stem_weight_gradient_vs_fp64(pkg, cuda):
    """The recompute path's stem weight gradient, formed through the
    BN-backward identity dW = k1 (dZ^T im - m1 sum im - m2 xhat^T im), against
    an fp64 recomputation from the same stored dZ (UNET_STEM_KEEP=1) and the
    conv output y0 recomputed in fp64 from the same bf16 image and weights (the
    kernel normalises its fp32 y, not the bf16 y0 it stores for tests):
    dY = BN-backward(dZ) in fp64, then conv2d_weight(xq, dY) in fp64."""
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=5)
    xs, ms = pkg.synthetic_cells(2, 256, 256, seed=13)
    x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
    _, v, g = _run(pkg, sd, x, y, {"UNET_STEM_KEEP": "1"})
    wq = sd["input_conv.weight"].to(torch.bfloat16).double()
    y0 = torch.nn.functional.conv2d(x.cpu().to(torch.bfloat16).double(), wq, stride=2, padding=3)
    dz = v["d.x1"].double() * (v["x1"] > 0).double()
    n = y0.shape[0] * y0.shape[2] * y0.shape[3]
    mu = y0.mean((0, 2, 3), keepdim=True)
    inv = 1.0 / torch.sqrt(y0.var((0, 2, 3), unbiased=False, keepdim=True) + 1e-5)
    xhat = (y0 - mu) * inv
    k1 = sd["bn1.weight"].double().view(1, -1, 1, 1) * inv
    dy = k1 * (dz - dz.sum((0, 2, 3), keepdim=True) / n - xhat * (dz * xhat).sum((0, 2, 3), keepdim=True) / n)
    xq = x.cpu().to(torch.bfloat16).double()
    dw = torch.nn.grad.conv2d_weight(xq, sd["input_conv.weight"].shape, dy, stride=2, padding=3)
    e = _rel(g["input_conv.weight"], dw)
    print(f"input_conv.weight vs fp64 from stored dZ: rel {e:.2e}")
    assert e <= W64_TOL
