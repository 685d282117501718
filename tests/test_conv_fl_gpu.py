"""Single-op parity of the full-line halo conv (conv3x3_fl_kernel, conv_fl.hip)
through its C-ABI entry unet_conv3x3_fl, against torch fp32 on the same bf16
operands (CPU reference).

conv3x3_fl_kernel runs every 3x3 / stride-1 conv with C >= 128 that fills the
chip -- the enc2 / enc3 BasicBlocks and decoder4 / decoder3 of the reference
(advanced_models.py:84-87,197-205) -- forward AND data gradient, ~23 % of the
step's GPU time.  The model-level routing and wiring at the
bench's own 16 x 512^2 workload are in test_fl_routing_gpu.py; this file reaches
the cases the model does not pin separately:
  * C = 256 / 512 (enc3 / decoder4 widths) and ragged maps (W != H);
  * every epilogue instance: forward plain / bias / BN statistics / addend
    (run-time flags); data gradient plain / addend / fused BN backward with and
    without addend / the two-BN (downsample block) epilogue;
  * the persistent multi-item path: the grid is capped (`grid` argument) so
    each block runs 2..8 work items, with the epilogue of item i beside item
    i+1's first sub-stage and the BN sums carried across items.
Tolerance (as test_kernels_gpu.py): bf16 outputs after fp32 accumulation,
|err| <= 1e-2 * max|ref| + 1e-2 * |ref| elementwise; BN sums of the stored
bf16 values relative 1e-4 (fp32 per-thread partials, fp64 across blocks)."""
import importlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

PK_CONV_FWD_CH, PK_CONV_DGRAD_CH = 5, 6
REP = 16  # kStatRep: BN sums are [16][2][C] replicas


@pytest.fixture(scope="module")
def L(pkg):
    return importlib.import_module("image-segmentation-project_amd._lib").load()


def S():
    return torch.cuda.current_stream().cuda_stream


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2)


def bf(t):
    return t.to(torch.bfloat16)


def close(got, ref, rel=1e-2):
    got, ref = got.float().cpu(), ref.float().cpu()
    tol = rel * ref.abs().max().item() + rel * ref.abs()
    err = (got - ref).abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} / {ref.numel()} elements off; max err {err.max().item():.4g} (ref max {ref.abs().max().item():.4g})"


def pack_ch(L, w, kind):
    """chunk-major pack of a forward weight w [Co][Ci][3][3]."""
    Co, Ci = w.shape[:2]
    dst = torch.empty(w.numel(), dtype=torch.bfloat16, device="cuda")
    assert L.unet_pack_weight(w.data_ptr(), dst.data_ptr(), kind, Co, Ci, 3, 3, S()) == 0, L.unet_last_error()
    return dst


def fl(L, x, wch, N, H, W, C, Co, mode, grid=0, bias=None, add=None, stats=None, bb=None):
    y = torch.empty(N, H, W, Co, dtype=torch.bfloat16, device="cuda")
    p = lambda t: 0 if t is None else t.data_ptr()
    ld = lambda t: 0 if t is None else t.shape[-1]
    bb = bb or {}
    rc = L.unet_conv3x3_fl(p(x), x.shape[-1], p(wch), p(y), Co, p(bias), p(add), ld(add), p(stats),
                           p(bb.get("act")), ld(bb.get("act")), p(bb.get("y")), ld(bb.get("y")),
                           p(bb.get("mean")), p(bb.get("invstd")), p(bb.get("y2")), ld(bb.get("y2")),
                           p(bb.get("mean2")), p(bb.get("invstd2")), p(bb.get("sums")), p(bb.get("sums2")),
                           N, H, W, C, Co, mode, grid, S())
    assert rc == 0, L.unet_last_error()
    return y


# N, C, H, W, Co, grid cap (0 = one block per CU)
CASES = [
    (2, 256, 32, 32, 256, 0),     # enc3 width, one item per block
    (2, 256, 32, 32, 256, 8),     # 4 items per block (ncb = 4: grid 8)
    (4, 512, 16, 16, 512, 16),    # decoder4.0-like C = 512, 2 items per block
    (1, 128, 32, 48, 128, 2),     # ragged map, 6 items per block
    (2, 128, 64, 64, 128, 0),     # enc2 geometry at batch 2
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("epi", ["plain", "bias_stats", "stats", "bias_add"])
def test_fl_forward(L, case, epi, cuda):
    N, C, H, W, Co, grid = case
    g = torch.Generator().manual_seed(11)
    x = bf(torch.randn(N, C, H, W, generator=g))
    w = torch.randn(Co, C, 3, 3, generator=g) / (C * 9) ** 0.5
    b = torch.randn(Co, generator=g) if "bias" in epi else None
    add = bf(torch.randn(N, Co, H, W, generator=g)) if "add" in epi else None
    ref = F.conv2d(x.float(), bf(w).float(), b, padding=1)
    if add is not None:
        ref = ref + add.float()
    stats = torch.zeros(REP * 2 * Co, dtype=torch.float64, device="cuda") if "stats" in epi else None
    xg, wg = nhwc(x).cuda(), w.cuda()
    wch = pack_ch(L, wg, PK_CONV_FWD_CH)
    bg = None if b is None else b.cuda()
    ag = None if add is None else nhwc(add).cuda()
    y = fl(L, xg, wch, N, H, W, C, Co, 0, grid, bias=bg, add=ag, stats=stats)
    torch.cuda.synchronize()
    close(nchw(y), ref)
    if stats is not None:
        s = stats.cpu().view(REP, 2, Co).sum(0)
        # sums of the fp32 values before the bf16 store
        torch.testing.assert_close(s[0], ref.double().sum((0, 2, 3)), rtol=1e-3,
                                   atol=1e-3 * ref.abs().max().item() * (N * H * W) ** 0.5)
        torch.testing.assert_close(s[1], ref.double().pow(2).sum((0, 2, 3)), rtol=2e-3, atol=1.0)


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("epi", ["plain", "add", "fbwd", "fbwd_add", "two"])
def test_fl_dgrad(L, case, epi, cuda):
    """Data gradient dX = conv2d_input(dY, w) of a forward conv w [C][Co][3][3]
    (this op's C = the forward's output channels): the dgrad pack (kind 6) and
    every training-step epilogue of the kernel."""
    N, C, H, W, Co, grid = case
    g = torch.Generator().manual_seed(12)
    w = torch.randn(C, Co, 3, 3, generator=g) / (Co * 9) ** 0.5   # forward Co = C here, forward Ci = Co
    dy = bf(torch.randn(N, C, H, W, generator=g))
    add = bf(torch.randn(N, Co, H, W, generator=g)) if "add" in epi else None
    da = torch.nn.grad.conv2d_input((N, Co, H, W), bf(w).float(), dy.float(), padding=1)
    if add is not None:
        da = da + add.float()
    fused = epi in ("fbwd", "fbwd_add", "two")
    bb = {}
    if fused:
        yraw = bf(torch.randn(N, Co, H, W, generator=g))
        act = bf(torch.relu(torch.randn(N, Co, H, W, generator=g)))   # ~half the mask zero
        mean, invstd = torch.randn(Co, generator=g) * 0.1, torch.rand(Co, generator=g) + 0.5
        bb = {"act": nhwc(act).cuda(), "y": nhwc(yraw).cuda(), "mean": mean.cuda(), "invstd": invstd.cuda(),
              "sums": torch.zeros(REP * 2 * Co, dtype=torch.float64, device="cuda")}
        if epi == "two":
            yraw2 = bf(torch.randn(N, Co, H, W, generator=g))
            mean2, invstd2 = torch.randn(Co, generator=g) * 0.1, torch.rand(Co, generator=g) + 0.5
            bb.update({"y2": nhwc(yraw2).cuda(), "mean2": mean2.cuda(), "invstd2": invstd2.cuda(),
                       "sums2": torch.zeros(REP * 2 * Co, dtype=torch.float64, device="cuda")})
        ref = da * (act.float() > 0).float()
    else:
        ref = da
    wch = pack_ch(L, w.cuda(), PK_CONV_DGRAD_CH)
    dyg = nhwc(dy).cuda()
    ag = None if add is None else nhwc(add).cuda()
    out = fl(L, dyg, wch, N, H, W, C, Co, 1, grid, add=ag, bb=bb)
    torch.cuda.synchronize()
    close(nchw(out), ref)
    if fused:
        dz = nchw(out).double().cpu()   # the sums are of the STORED bf16 dZ (bn_bwd_reduce_kernel's view)
        assert bool((dz[act == 0] == 0).all())   # the ReLU mask of the fused BN backward
        s = bb["sums"].cpu().view(REP, 2, Co).sum(0)
        xhat = (yraw.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
        r0, r1 = dz.sum((0, 2, 3)), (dz * xhat).sum((0, 2, 3))
        sc = dz.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(s[0], r0, rtol=1e-4, atol=1e-5 * sc)
        torch.testing.assert_close(s[1], r1, rtol=1e-4, atol=1e-5 * sc * xhat.abs().max().item())
        if epi == "two":
            s2 = bb["sums2"].cpu().view(REP, 2, Co).sum(0)
            xhat2 = (yraw2.double() - mean2.double().view(1, -1, 1, 1)) * invstd2.double().view(1, -1, 1, 1)
            torch.testing.assert_close(s2[1], (dz * xhat2).sum((0, 2, 3)), rtol=1e-4,
                                       atol=1e-5 * sc * xhat2.abs().max().item())
            assert s2[0].abs().max().item() == 0.0   # only the dZ*xhat2 half is used


def test_fl_grid_cap_is_bit_identical(L, cuda):
    """The persistent multi-item path computes each work item exactly as the
    one-item-per-block launch does (same MFMA order per item): outputs are
    bit-identical whatever the grid."""
    N, C, H, W, Co = 2, 256, 32, 32, 128
    g = torch.Generator().manual_seed(13)
    x = nhwc(bf(torch.randn(N, C, H, W, generator=g))).cuda()
    wch = pack_ch(L, (torch.randn(Co, C, 3, 3, generator=g) / (C * 9) ** 0.5).cuda(), PK_CONV_FWD_CH)
    outs = [fl(L, x, wch, N, H, W, C, Co, 0, grid) for grid in (0, 2, 4, 6)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_fl_rejects_uncovered_shapes(L, cuda):
    """The kernel covers C % 128 == 0, Cout % 64 == 0 and 16-multiples of H, W;
    anything else is refused before a launch (no silent routing elsewhere)."""
    x = torch.zeros(1, 16, 16, 192, dtype=torch.bfloat16, device="cuda")
    w = torch.zeros(64 * 192 * 9, dtype=torch.bfloat16, device="cuda")
    for (H, W, C, Co) in [(16, 16, 192, 64), (16, 16, 128, 96), (24, 16, 128, 64), (16, 8, 128, 64)]:
        rc = L.unet_conv3x3_fl(x.data_ptr(), C, w.data_ptr(), x.data_ptr(), Co, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               0, 0, 0, 0, 1, H, W, C, Co, 0, 0, S())
        assert rc != 0
