"""HiRes configuration (BASELINE.json configs[3]: 1024x1024 tiles, batch 4) on
the HIP path, checked against the oracle on the same seeded inputs.

Tolerances are the end-to-end ones of test_model_gpu.py (bf16 path vs the fp32
reference; a random-init BN ResNet amplifies rounding with depth):
  train logits ||d||/||ref|| <= 0.10; masks agree on >= 95 % of pixels and are
  bit-exact where |logit_ref| > 1; BCE/Dice/Combo loss relative 1e-3;
  calculate_metrics of the HIP logits bit-exact vs. the oracle's aggregation of
  the same logits, and within 1e-3 of the oracle's metrics on its own logits
  (north-star mIoU bar); every gradient finite and one Adam step changes the loss.
"""
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
THR = 8.94069742685133e-08


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_hires_1024_batch4_train_step(pkg, cuda):
    torch.set_num_threads(min(16, torch.get_num_threads()))
    xs, ms = pkg.synthetic_cells(4, 1024, 1024, seed=1234)
    x, y = torch.from_numpy(xs), torch.from_numpy(ms)
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=0)
    ref.load_state_dict(sd)
    ref.train()
    with torch.no_grad():
        ref_logits = ref(x)
    m = pkg.UNetWithBackbone(n_classes=1, backbone="resnet34", pretrained=False, use_attention=False)
    m.load_state_dict(sd)
    m = m.cuda().train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    logits = m(x.cuda())
    assert logits.shape == (4, 1, 1024, 1024)
    e = _rel(logits, ref_logits)
    print(f"1024^2 train logits rel err {e:.3e}")
    assert e <= 0.10
    lg = logits.detach().cpu()
    assert (lg >= THR).eq(ref_logits >= THR).float().mean() >= 0.95
    far = ref_logits.abs() > 1.0
    assert torch.equal((lg >= THR)[far], (ref_logits >= THR)[far])
    for name in ("bce", "dice", "combo"):
        v = pkg.get_loss_function({"loss_fn": name})(logits, y.cuda()).item()
        ref_v = oracle.get_loss_function({"loss_fn": name})(ref_logits, y).item()
        assert abs(v - ref_v) <= 1e-3 * abs(ref_v), (name, v, ref_v)
    # metric aggregation of the HIP logits: bit-exact vs the oracle on the same logits
    got = pkg.calculate_metrics_from_logits(logits.detach(), y.cuda())
    want = oracle.calculate_metrics(torch.sigmoid(lg), y)
    for k in want:
        assert got[k] == pytest.approx(want[k], abs=0.0, rel=1e-12), k
    # north-star bar: mIoU of the HIP path within 1e-3 of the reference path's
    want_ref = oracle.calculate_metrics(torch.sigmoid(ref_logits), y)
    print(f"1024^2 IoU hip {got['iou']:.6f} ref {want_ref['iou']:.6f}")
    for k in want_ref:
        assert abs(got[k] - want_ref[k]) <= 1e-3, k
    loss = pkg.get_loss_function({"loss_fn": "bce"})(logits, y.cuda())
    opt.zero_grad()
    loss.backward()
    for k, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k
    opt.step()
    loss2 = pkg.get_loss_function({"loss_fn": "bce"})(m(x.cuda()), y.cuda()).item()
    assert loss2 != loss.item() and torch.isfinite(torch.tensor(loss2))
