"""In-kernel s_memtime breakdown of the halo-streamed conv (debug build with
HS_TIMING): per-stage cycles, epilogue and stats cycles, block spread.
usage: UNET_HIP_LIB=<timing build> python scripts/hs_timing.py"""
import ctypes
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
importlib.import_module("image-segmentation-project_amd")
L = importlib.import_module("image-segmentation-project_amd._lib").load()
lib = ctypes.CDLL(importlib.import_module("image-segmentation-project_amd._lib").LIB_PATH)
N = 16
S = lambda: torch.cuda.current_stream().cuda_stream
for name, C, Co, H in [("enc3", 256, 256, 32), ("enc4", 512, 512, 16), ("dec3.0", 256, 128, 64)]:
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    y = torch.empty(N, H, H, Co, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(Co * 9 * C, device="cuda").to(torch.bfloat16)
    b = torch.zeros(Co, device="cuda")
    st = torch.zeros(16 * 2 * Co, device="cuda", dtype=torch.float64)
    a = (x.data_ptr(), C, w.data_ptr(), y.data_ptr(), Co, b.data_ptr(), 0, 0, st.data_ptr(), N, H, H, C, H, H, Co, 3, 3, 1, 1, 0)
    for _ in range(3):
        L.unet_conv_fwd(*a, S())
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (1024 * 32))()
    lib.unet_debug_timing(buf, 1024 * 32)
    d = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 32).astype(np.int64)
    nb = int((d[:, 20] > 0).sum())
    d = d[:nb]
    KC = C // 32
    st_ = np.diff(d[:, 2:2 + min(KC, 16)], axis=1)
    print(f"{name}: blocks {nb}  prologue(start->stage0) {np.median(d[:, 2] - d[:, 1]):.0f} cyc  "
          f"stage median {np.median(st_):.0f} (min {st_.min()} max {st_.max()})  last stage->loop end "
          f"{np.median(d[:, 18] - d[:, 1 + min(KC, 16)]):.0f}  epi store {np.median(d[:, 19] - d[:, 18]):.0f}  "
          f"stats {np.median(d[:, 20] - d[:, 19]):.0f}  total {np.median(d[:, 20] - d[:, 1]):.0f} cyc")
    rs, re_ = d[:, 0], d[:, 21]
    print(f"   realtime(100MHz): block start spread {(rs.max() - rs.min()) / 100:.2f} us, "
          f"block dur median {np.median(re_ - rs) / 100:.2f} us, kernel span {(re_.max() - rs.min()) / 100:.2f} us")
