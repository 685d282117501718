import sys
import torch
a, b = torch.load(sys.argv[1]), torch.load(sys.argv[2])
worst = sorted(((((a[k] - b[k]).norm() / b[k].norm().clamp_min(1e-30)).item(), k) for k in a), reverse=True)
for e, k in worst[:12]:
    print(f"{k:40s} {e:.3e}")
