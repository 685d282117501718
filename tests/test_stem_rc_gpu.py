"""The stem by recompute (csrc/stem_rc.hip, the default for stem rows of up
to 256 pixels) against the stored-y0 stem path (UNET_STEM_RC=0: stem_fwd +
bn_relu_maxpool_fwd + maxpool_bwd + BN-fused stem_wgrad) on the same inputs
and weights (resnet34 stem, advanced_models.py:76-83).

The two paths compute y with the same MFMA sequence, but the BN batch sums
are accumulated in another order (fp32 partials -> fp64), so scale/shift may
differ in the last bit and a few bf16 activations round the other way; and
the recompute path forms the stem weight gradient through the BN-backward
identity dW = k1 (dZ^T im - m1 sum im - m2 xhat^T im) instead of rounding
dY = k1 (dZ - m1 - m2 xhat) to bf16 first.  Bars: forward activations (x1,
pooled p0) relative L2 <= 1e-3 with >= 99 % of elements bit-equal and the
argmax index equal wherever the inputs are; every parameter gradient relative
L2 <= 1e-2 (input_conv.weight, the one computed differently: <= 2e-2); the
recompute path's backward is bit-reproducible.  The teacher-forced rows of
test_wiring_gpu.py (UNET_STEM_KEEP=1) pin the recompute path's dZ, bn1 and
input_conv gradients against fp32 recomputations at 2e-2.
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
        assert e <= 1e-3 and same >= 0.99, (k, e, same)
    print("logits rel", _rel(o_rc, o_st))
    assert _rel(o_rc, o_st) <= 1e-2
    worst = sorted(((_rel(g_rc[k], g_st[k]), k) for k in g_st if g_st[k].norm() > 0), reverse=True)[:6]
    print("largest gradient differences:", [(k, f"{e:.2e}") for e, k in worst])
    for e, k in worst:
        assert e <= (2e-2 if k == "input_conv.weight" else 1e-2), (k, e)
    # bit-reproducible: the same step again on the recompute path
    o2, v2, g2 = _run(pkg, sd, x, y, {"UNET_STEM_RC": "1"})
    assert torch.equal(o2, o_rc)
    for k in g_rc:
        assert torch.equal(g2[k], g_rc[k]), k
