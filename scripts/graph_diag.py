"""Diagnose HIP-graph capture of the train step after eager steps.
usage: python scripts/graph_diag.py {torch|fused} {eager_steps} {del_loss 0|1}"""
import importlib, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("image-segmentation-project_amd")
which, neager, dl = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cuda = torch.device("cuda")
torch.manual_seed(0)
m = pkg.UNetWithBackbone(pretrained=False, use_attention=False).to(cuda).train()
xs, ms = pkg.synthetic_cells(2, 64, 64, seed=5)
x, y = torch.from_numpy(xs).to(cuda), torch.from_numpy(ms).to(cuda)
crit = pkg.get_loss_function({"loss_fn": "bce"})
opt = pkg.optim.Adam(m.parameters(), lr=1e-3) if which == "fused" else torch.optim.Adam(m.parameters(), lr=1e-3, capturable=True)
for _ in range(neager):
    loss = crit(m(x), y)
    opt.zero_grad()
    loss.backward()
    opt.step()
if dl and neager:
    del loss
torch.cuda.synchronize()
print("eager done", flush=True)
step = pkg.GraphedTrainStep(m, crit, opt, x, y)
print("captured", flush=True)
print([round(float(step()[1]), 5) for _ in range(5)], flush=True)
