"""Micro-timing of the weight-stationary up-conv (unet_convt2x2) at the Base
config's upconv2 / upconv1 shapes: forward into a dense buffer and into a
concat slice, data gradient plain / fused, against a device copy of the same
bytes (the achievable HBM rate for this traffic).  HIP events, median of 50."""
import ctypes
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
L = importlib.import_module("image-segmentation-project_amd._lib").load()


def S():
    return torch.cuda.current_stream().cuda_stream


def t_ms(fn, it=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(it):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    grid = int(os.environ.get("CT_GRID", "0"))
    for (Ci, Co, H) in [(128, 64, 64), (64, 32, 128)]:
        N = 16
        x = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
        w = torch.randn(Ci, Co, 2, 2, device="cuda") / Ci ** 0.5
        wp = torch.empty(w.numel(), dtype=torch.bfloat16, device="cuda")
        wd = torch.empty(w.numel(), dtype=torch.bfloat16, device="cuda")
        assert L.unet_pack_weight(w.data_ptr(), wp.data_ptr(), 2, Co, Ci, 2, 2, S()) == 0
        assert L.unet_pack_weight(w.data_ptr(), wd.data_ptr(), 3, Co, Ci, 2, 2, S()) == 0
        b = torch.zeros(Co, device="cuda")
        for ld in (Co, 2 * Co, Co + 64):
            y = torch.empty(N, 2 * H, 2 * H, ld, dtype=torch.bfloat16, device="cuda")
            f = lambda: L.unet_convt2x2(x.data_ptr(), Ci, wp.data_ptr(), y.data_ptr(), ld, b.data_ptr(), 0, 0, 0, 0,
                                        0, 0, 0, 0, N, H, H, Ci, Co, 0, grid, S())
            ms = t_ms(f)
            mb = (x.numel() + N * 4 * H * H * Co) * 2 / 1e6
            print(f"fwd  Ci {Ci:3d} Co {Co:3d} H {H:3d} ldy {ld:3d}: {ms * 1e3:7.1f} us  {mb:6.1f} MB  {mb / ms / 1e3:5.2f} TB/s")
        dy = torch.randn(N, 2 * H, 2 * H, Co, device="cuda").to(torch.bfloat16)
        dx = torch.empty(N, H, H, Ci, dtype=torch.bfloat16, device="cuda")
        act = torch.randn(N, H, H, Ci, device="cuda").clamp_min(0).to(torch.bfloat16)
        yr = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
        mean = torch.zeros(Ci, device="cuda")
        inv = torch.ones(Ci, device="cuda")
        sums = torch.zeros(16 * 2 * Ci, dtype=torch.float64, device="cuda")
        bacc = torch.zeros(16 * Co, dtype=torch.float64, device="cuda")
        for fused in (False, True):
            a_ = (act.data_ptr(), Ci, yr.data_ptr(), Ci, mean.data_ptr(), inv.data_ptr(), sums.data_ptr()) if fused \
                else (0, 0, 0, 0, 0, 0, 0)
            f = lambda: L.unet_convt2x2(dy.data_ptr(), Co, wd.data_ptr(), dx.data_ptr(), Ci, 0, *a_, bacc.data_ptr(),
                                        N, H, H, Ci, Co, 1, grid, S())
            ms = t_ms(f)
            mb = (dy.numel() + dx.numel() * (3 if fused else 1)) * 2 / 1e6
            print(f"dgrad Ci {Ci:3d} Co {Co:3d} H {H:3d} fused {int(fused)}: {ms * 1e3:7.1f} us  {mb:6.1f} MB  {mb / ms / 1e3:5.2f} TB/s")
        # reference: a device copy moving the forward's bytes (read x-sized + write y-sized)
        src = torch.empty(N * 4 * H * H * Co, dtype=torch.bfloat16, device="cuda")
        dst = torch.empty_like(src)
        ms = t_ms(lambda: dst.copy_(src))
        mb = src.numel() * 4 / 1e6
        print(f"copy {src.numel() * 2 / 1e6:6.1f} MB -> {ms * 1e3:7.1f} us  {mb / ms / 1e3:5.2f} TB/s (r+w)")


if __name__ == "__main__":
    main()
