"""Time every implicit-GEMM tile configuration on the U-Net's conv shapes
(Base config, N=16) in one process, interleaved (cdna_hip_programming.md §5.4
rule 24).  Prints, per shape and mode, the median us of each config and the
best one.  usage: python scripts/tune_conv.py [--reps 5]"""
import argparse
import importlib
import sys

import torch

sys.path.insert(0, ".")
importlib.import_module("image-segmentation-project_amd")
L = importlib.import_module("image-segmentation-project_amd._lib").load()

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--n", type=int, default=16)
ap.add_argument("--cfgs", type=str, default="0,1,2,3,4,5,6,7,8,9,10,11,12,13,14")
ap.add_argument("--only", type=str, default="", help="comma list of shape names to run")
ap.add_argument("--modes", type=str, default="0,1")
ap.add_argument("--epi", action="store_true", help="forward with bias + BN statistics epilogue")
args = ap.parse_args()
N = args.n
CFGS = [int(c) for c in args.cfgs.split(",")]
S = lambda: torch.cuda.current_stream().cuda_stream

# (name, C_in, C_out, H_in, R, stride, pad) forward geometry of the conv
SHAPES = [
    ("enc1_3x3", 64, 64, 128, 3, 1, 1),
    ("enc2_3x3", 128, 128, 64, 3, 1, 1),
    ("enc3_3x3", 256, 256, 32, 3, 1, 1),
    ("enc4_3x3", 512, 512, 16, 3, 1, 1),
    ("dec4.0", 512, 256, 32, 3, 1, 1),
    ("dec3.0", 256, 128, 64, 3, 1, 1),
    ("dec2.0", 128, 64, 128, 3, 1, 1),
    ("dec1.0", 96, 32, 256, 3, 1, 1),
    ("dec1.3", 32, 32, 256, 3, 1, 1),
    ("enc2.0_s2", 64, 128, 128, 3, 2, 1),
    ("enc3.0_s2", 128, 256, 64, 3, 2, 1),
    ("enc4.0_s2", 256, 512, 32, 3, 2, 1),
    # ConvTranspose k2s2 data gradients = k2s2 convs of dY (dY channels in, X channels out)
    ("up1_dgrad", 32, 64, 256, 2, 2, 0),
    ("up2_dgrad", 64, 128, 128, 2, 2, 0),
]


def run(mode, C, Co, H, R, st, pad):
    """mode 0: forward conv; mode 1: dgrad (transposed gather) of that conv;
    mode 2: weight gradient (fp32 atomics into dW, no split-K slab)."""
    P = (H + 2 * pad - R) // st + 1
    if mode == 2:
        dy = torch.randn(N, P, P, Co, device="cuda").to(torch.bfloat16)
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(Co * R * R * C, device="cuda")
        args_ = (dy.data_ptr(), Co, x.data_ptr(), C, dw.data_ptr(), N, H, H, C, P, P, Co, R, R, st, pad, 0)
        return args_, 2.0 * N * P * P * Co * C * R * R, (dy, dw, x)
    if mode == 0:
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        y = torch.empty(N, P, P, Co, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(Co * R * R * C, device="cuda").to(torch.bfloat16)
        b = torch.zeros(Co, device="cuda")
        stats = torch.zeros(16 * 2 * Co, device="cuda", dtype=torch.float64)
        bp, sp = (b.data_ptr(), stats.data_ptr()) if args.epi else (0, 0)
        args_ = (x.data_ptr(), C, w.data_ptr(), y.data_ptr(), Co, bp, 0, 0, sp, N, H, H, C, P, P, Co, R, R, st, pad, 0)
        flops = 2.0 * N * P * P * Co * C * R * R
        keep = (x, y, w, b, stats)
        return args_, flops, keep
    else:
        x = torch.randn(N, P, P, Co, device="cuda").to(torch.bfloat16)
        y = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(Co * R * R * C, device="cuda").to(torch.bfloat16)
        args_ = (x.data_ptr(), Co, w.data_ptr(), y.data_ptr(), C, 0, 0, 0, 0, N, P, P, Co, H, H, C, R, R, st, pad, 1)
        flops = 2.0 * N * P * P * Co * C * R * R
    keep = (x, y, w)
    return args_, flops, keep


e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ONLY = [o for o in args.only.split(",") if o]
for name, C, Co, H, R, st, pad in SHAPES:
    if ONLY and name not in ONLY:
        continue
    for mode in [int(m) for m in args.modes.split(",")]:
        a, flops, keep = run(mode, C, Co, H, R, st, pad)
        fn = L.unet_conv_wgrad if mode == 2 else L.unet_conv_fwd
        times = {c: [] for c in CFGS}
        y = keep[1]
        L.unet_set_conv_config(0)
        fn(*a, S())
        y_ref = y.clone()
        bad = []
        for c in CFGS:
            y.zero_()
            L.unet_set_conv_config(c)
            if fn(*a, S()) == 0 and not torch.equal(y, y_ref):
                bad.append((c, (y.float() - y_ref.float()).abs().max().item()))
        if bad:
            print(f"{name} mode {mode}: configs differ from auto: {bad}", flush=True)
        for rep in range(args.reps):
            for c in CFGS:
                L.unet_set_conv_config(c)
                if fn(*a, S()) != 0:
                    times[c] = None
                    continue
                if times[c] is None:
                    continue
                e0.record()
                for _ in range(5):
                    fn(*a, S())
                e1.record()
                torch.cuda.synchronize()
                times[c].append(e0.elapsed_time(e1) / 5 * 1e3)
        L.unet_set_conv_config(0)
        res = {c: sorted(t)[len(t) // 2] for c, t in times.items() if t}
        best = min(res, key=res.get)
        line = " ".join(f"{c}:{res[c]:.0f}" for c in sorted(res))
        print(f"{name:10s} {['fwd', 'dgrad', 'wgrad'][mode]:5s} best cfg {best:2d} {res[best]:7.1f}us "
              f"{flops / res[best] / 1e6:6.0f} TF | auto {res.get(0, 0):.0f}us | {line}", flush=True)
