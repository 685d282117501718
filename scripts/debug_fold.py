"""Bit-reproducibility probe of the enc2.0 conv1 weight gradient (two identical
backwards); prints the differing [co, ci, r, s] pattern."""
import importlib, sys, torch
sys.path.insert(0, ".")
pkg = importlib.import_module("image-segmentation-project_amd")
torch.manual_seed(0)
m = pkg.UNetWithBackbone(pretrained=False).cuda().train()
xs, ms = pkg.synthetic_cells(4, 128, 128, seed=12)
x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
crit = pkg.get_loss_function({"loss_fn": "bce"})
sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
runs = []
for _ in range(3):
    m.load_state_dict(sd)
    for p in m.parameters():
        p.grad = None
    crit(m(x), y).backward()
    torch.cuda.synchronize()
    runs.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
for k in runs[0]:
    for j in (1, 2):
        a, b = runs[0][k], runs[j][k]
        if not torch.equal(a, b):
            d = (a - b).abs()
            idx = (d > 0).nonzero()
            print(k, j, "ndiff", idx.shape[0], "of", a.numel(), "max", d.max().item(), "ref", a.abs().max().item())
            for dim in range(idx.shape[1]):
                print("   dim", dim, "values", torch.unique(idx[:, dim]).tolist()[:40])
print("done")
