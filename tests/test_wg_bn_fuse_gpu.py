"""The BN-backward apply (dY = A dZ + B y + C, bn_bwd_apply_kernel) run inside
the following 3x3 / stride-1 weight gradient (wgrad3x3_halo_kernel FUSE,
DESIGN.md §7e) against the separate apply pass it replaces: the dY side
product the dgrad reads, every later gradient tensor, every parameter gradient
(dgamma / dbeta included) and every BN buffer must be BIT-identical (the fused
staging evaluates the apply's expression with the apply's coefficients,
bn_bwd_apply_coef), at a size where enc1-3 and decoder2/3 take the fused path.
The fused path is opt-in (UNET_WG_BN=1): it measured slower than the apply
pass it replaces.  Without apply launches to ride on, deferred split-K
reductions run on their own, so this test also covers the slab-reuse ordering
in wgrad_and_reduce."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(pkg, sd, x, y, att):
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=att)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x)
    pkg.get_loss_function({"loss_fn": "bce"})(out, y).backward()
    torch.cuda.synchronize()
    views = {k: v.clone() for k, v in m._last_plan.tensor_views().items()}
    grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    bufs = {k: b.detach().clone() for k, b in m.named_buffers()}
    return out.detach().clone(), views, grads, bufs


@pytest.mark.parametrize("att", [False, True])
def test_wgrad_bn_fuse_bit_identical(pkg, cuda, monkeypatch, att):
    torch.manual_seed(0)
    sd = {k: v.detach().clone()
          for k, v in pkg.UNetWithBackbone(pretrained=False, use_attention=att).state_dict().items()}
    xs, ms = pkg.synthetic_cells(2, 256, 256, seed=23)
    x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
    # both runs on the per-layer weight-gradient kernels (the fused apply is
    # one of them; the default batched launch sums split partials differently)
    monkeypatch.setenv("UNET_WG_BATCH", "0")
    monkeypatch.setenv("UNET_WG_BN", "1")  # read when the native plan is created
    fused = _run(pkg, sd, x, y, att)
    monkeypatch.delenv("UNET_WG_BN")
    plain = _run(pkg, sd, x, y, att)
    assert torch.equal(fused[0], plain[0])
    dys = [k for k in plain[1] if k.endswith("d.y1") or k.endswith("d.y2")]
    assert len(dys) >= 20
    bad = []
    for k, v in plain[1].items():
        f = fused[1][k]
        if not torch.equal(f, v):
            d = (f.float() - v.float()).abs()
            bad.append((k, round(float((f != v).float().mean()), 4), float(d.nan_to_num(1e30).max()),
                        int(torch.isnan(f.float()).sum())))
    print("mismatching tensors (name, fraction, max |diff|, NaNs):", bad)
    assert not bad, bad
    gbad = [k for k, v in plain[2].items() if not torch.equal(fused[2][k], v)]
    print("mismatching gradients:", gbad)
    assert not gbad, gbad
    for k, v in plain[3].items():
        assert torch.equal(fused[3][k], v), k
