"""Wide U-Net (BASELINE.json configs[4]: every channel count x2, 128 -> 1024)
on the HIP path, checked against the oracle (``ReferenceUNet(width=2)``, the
reference topology of advanced_models.py:72-100,157-160 with doubled channels)
on the same seeded inputs and closed-form weights.

The HIP path computes in bf16 here (the configs[4] fp8 forward, ``fp8=True``,
is checked by test_fp8_gpu.py and, at its 16 x 512^2 workload, by
test_wide_fp8_full_gpu.py). Tolerances are the end-to-end ones of test_model_gpu.py:
  train logits ||d||/||ref|| <= 0.10; masks agree on >= 95 % of pixels and are
  bit-exact where |logit_ref| > 1; BCE loss relative 1e-3; every gradient
  finite; head gradients within relative L2 0.10.  Every other op and gradient
  is checked teacher-forced at 2e-2 by test_wiring_gpu.py[wide].
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


def test_wide_width2_train_step(pkg, cuda):
    torch.set_num_threads(min(16, torch.get_num_threads()))
    n, s = 2, 256
    xs, ms = pkg.synthetic_cells(n, s, s, seed=1234)
    x, y = torch.from_numpy(xs), torch.from_numpy(ms)
    ref = oracle.ReferenceUNet(width=2)
    sd = oracle.closed_form_state_dict(ref, seed=0)
    ref.load_state_dict(sd)
    ref.train()
    ref_logits = ref(x)
    ref_loss = oracle.get_loss_function({"loss_fn": "bce"})(ref_logits, y)
    ref_loss.backward()
    ref_grads = {k: p.grad.detach().clone() for k, p in ref.named_parameters()}

    m = pkg.UNetWithBackbone(n_classes=1, backbone="resnet34", pretrained=False, use_attention=False, width=2)
    assert sum(p.numel() for p in m.parameters()) == sum(p.numel() for p in ref.parameters())
    m.load_state_dict(sd)
    m = m.cuda().train()
    logits = m(x.cuda())
    assert logits.shape == (n, 1, s, s)
    lg = logits.detach().cpu()
    rl = ref_logits.detach()
    e = _rel(lg, rl)
    print(f"width=2 train logits rel err {e:.3e}")
    assert e <= 0.10
    assert (lg >= THR).eq(rl >= THR).float().mean() >= 0.95
    far = rl.abs() > 1.0
    assert torch.equal((lg >= THR)[far], (rl >= THR)[far])
    loss = pkg.get_loss_function({"loss_fn": "bce"})(logits, y.cuda())
    assert abs(loss.item() - ref_loss.item()) <= 1e-3 * abs(ref_loss.item())
    loss.backward()
    params = dict(m.named_parameters())
    for k, p in params.items():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k
    # head gradients end to end (deeper ones are pinned per op, teacher-forced,
    # by test_wiring_gpu.py[wide]: a random-init BN ResNet amplifies bf16
    # rounding with depth, as test_model_gpu.py documents)
    for k in ("conv_final.weight", "conv_final.bias", "upconv0.weight", "upconv0.bias"):
        ge = _rel(params[k].grad, ref_grads[k])
        print(f"grad {k}: rel {ge:.3e}")
        assert ge <= 0.1, k
