"""In-kernel phase breakdown of every conv launch of one Base training step.

Runs with the debug library that carries the phase stamps (common.h TSTAMP):
  make -C image-segmentation-project_amd/csrc timing
  UNET_HIP_LIB=$PWD/image-segmentation-project_amd/libunet_hip_timing.so python scripts/conv_timing.py
Per launch: blocks, kernel span (s_memrealtime, 100 MHz), effective shader clock,
and the block-median cycles of each phase: prologue (start -> loop), per stage
or per tile, MFMA-loop tail, epilogue store, BN-statistics commit."""
import argparse
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--size", type=int, default=512)
ap.add_argument("--filter", default="")
ap.add_argument("--width", type=int, default=1)
args = ap.parse_args()
assert "timing" in os.environ.get("UNET_HIP_LIB", ""), "set UNET_HIP_LIB to libunet_hip_timing.so"
pkg = importlib.import_module("image-segmentation-project_amd")
torch.manual_seed(0)
m = pkg.UNetWithBackbone(pretrained=False, use_attention=False, width=args.width).cuda().train()
xs, ms = pkg.synthetic_cells(args.batch, args.size, args.size, seed=1234)
x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
crit = pkg.BCELoss()


def step():
    out = m(x)
    loss = crit(out, y)
    m.zero_grad()
    loss.backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
plan = m._last_plan
lib = plan.lib
KL, KB, KS = 320, 1024, 32
assert lib.unet_timing_enable(plan.handle, 1) == 0
step()
torch.cuda.synchronize()
buf = np.zeros(KL * KB * KS, dtype=np.uint64)
names = ctypes.create_string_buffer(1 << 16)
n = lib.unet_timing_read(plan.handle, buf.ctypes.data, KL, names, 1 << 16)
lib.unet_timing_enable(plan.handle, 0)
names = names.value.decode().splitlines()
d = buf.reshape(KL, KB, KS).astype(np.int64)
tot_span = 0.0
for i in range(n):
    nm = names[i]
    if args.filter and args.filter not in nm:
        continue
    t = d[i]
    live = t[:, 0] > 0
    nb = int(live.sum())
    if nb == 0:
        continue
    t = t[live]
    rt0, rt1 = t[:, 30], t[:, 31]
    ok = rt1 > 0
    span = (rt1[ok].max() - rt0.min()) / 100.0 if ok.any() else float("nan")  # us
    tot_span += span
    dur_rt = np.median((rt1 - rt0)[ok]) / 100.0 if ok.any() else float("nan")
    last = np.where(t[:, 21] > 0, t[:, 21], t[:, 20])
    if (t[:, 22] > 0).any():
        last = np.where(t[:, 22] > 0, t[:, 22], last)
    cyc = np.median(last - t[:, 0])
    clk = cyc / dur_rt / 1e3 if dur_rt == dur_rt and dur_rt > 0 else float("nan")
    stages = [k for k in range(2, 20) if (t[:, k] > 0).mean() > 0.5]
    parts = [f"pro {np.median(t[:, 1] - t[:, 0]):.0f}"]
    if stages:
        st = np.diff(t[:, [1] + stages], axis=1)
        parts.append(f"st[{len(stages)}] " + " ".join(f"{v:.0f}" for v in np.median(st, axis=0)))
        parts.append(f"tail {np.median(t[:, 20] - t[:, stages[-1]]):.0f}")
    if (t[:, 21] > 0).any():
        parts.append(f"epi {np.median(t[:, 21] - t[:, 20]):.0f}")
    if (t[:, 22] > 0).any():
        parts.append(f"stats {np.median(t[:, 22] - t[:, 21]):.0f}")
    if (t[:, 23] > 0).mean() > 0.5:  # loader-wave stamps (conv3x3_fl_kernel)
        ld = lambda k, j: np.median(t[:, k] - t[:, j])
        parts.append(f"ld: issue0 {ld(24, 23):.0f} land0 {ld(25, 24):.0f}")
        if (t[:, 27] > 0).mean() > 0.5:
            parts.append(f"land1 {ld(27, 26):.0f}")
        if (t[:, 28] > 0).mean() > 0.5:
            parts.append(f"Z->epi-end {ld(21, 28):.0f}")
    start_spread = (rt0.max() - rt0.min()) / 100.0
    print(f"{nm:34s} blk {nb:4d} span {span:6.1f}us blk-dur {dur_rt:5.1f}us start-spread {start_spread:4.1f}us "
          f"clk {clk:4.2f}GHz | " + " | ".join(parts), flush=True)
print(f"sum of spans {tot_span:.1f} us over {n} launches")
