"""(Test tooling, not collected by pytest: may import the oracle.)  Measure end-to-end deviation of the HIP path from the fp32 oracle at several
input sizes (prints one line per size).  Used to state the tolerances of
tests/test_model_gpu.py."""
import importlib
import sys

import torch

sys.path.insert(0, ".")
import oracle  # noqa: E402

pkg = importlib.import_module("image-segmentation-project_amd")


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


for (n, h) in [(4, 64), (4, 128), (2, 256), (4, 256)]:
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=0)
    ref.load_state_dict(sd)
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=False)
    m.load_state_dict(sd)
    m = m.cuda().train()
    xs, ms = pkg.synthetic_cells(n, h, h, seed=1234)
    x, y = torch.from_numpy(xs), torch.from_numpy(ms)
    ref.train()
    lr = ref(x)
    l_ref = oracle.bce_with_logits(lr, y)
    l_ref.backward()
    lo = m(x.cuda())
    l_hip = pkg.BCELoss()(lo, y.cuda())
    l_hip.backward()
    gp = dict(m.named_parameters())
    gerr = sorted(rel(gp[k].grad, p.grad) for k, p in ref.named_parameters()
                  if not (k.startswith("decoder") and k.endswith("bias") and (".0." in k or ".3." in k)))
    mask_ref = lr.detach() >= 8.94069742685133e-08
    mask_hip = lo.detach().cpu() >= 8.94069742685133e-08
    iou_ref = oracle.calculate_metrics(torch.sigmoid(lr.detach()), y)["iou"]
    iou_hip = pkg.calculate_metrics_from_logits(lo.detach(), y.cuda())["iou"]
    print(f"N={n} H={h}: logits {rel(lo, lr.detach()):.3e} loss {l_hip.item():.6f} vs {l_ref.item():.6f} "
          f"grad median {gerr[len(gerr) // 2]:.3e} max {gerr[-1]:.3e} mask-agree {(mask_ref == mask_hip).float().mean():.5f} "
          f"iou {iou_hip:.6f} vs {iou_ref:.6f}", flush=True)
    m.eval(); ref.eval()
    with torch.no_grad():
        print(f"   eval logits {rel(m(x.cuda()), ref(x)):.3e}", flush=True)
