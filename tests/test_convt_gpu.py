"""Single-op parity of the weight-stationary ConvTranspose2d(k2, s2)
(convt2x2_kernel, convt.hip) through its C-ABI entry unet_convt2x2, against
torch fp32 on the same bf16 operands (CPU reference).

The kernel runs the narrow decoder up-convs of the reference
(advanced_models.py:96-99: upconv2 128->64, upconv1 64->32; Wide upconv1
128->64), forward and data gradient; the model-level wiring is teacher-forced
in test_wiring_gpu.py (dec*.up, the convT dgrad rows, g upconv*.bias) and the
routing at the bench workload in test_fl_routing_gpu.py.  Here:
  * every (Ci, Co) the kernel takes, ragged maps (W != H), batch 1-3;
  * forward into a concat slice (ld > Co, channel offset) with bias, the other
    channels untouched;
  * data gradient from a concat slice of dY, plain and with the fused BN(+ReLU)
    backward (dZ stored under the forward output's ReLU mask, sum dZ and
    sum dZ * xhat of the stored bf16 dZ into [16][2][Ci] replicas) and the
    up-conv's bias gradient (sum of dY into [16][Co] replicas);
  * grid caps (a block walks many pixel groups): results bit-identical to the
    production grid for the stored tensors.
Tolerances as test_conv_fl_gpu.py: bf16 outputs after fp32 accumulation,
|err| <= 1e-2 * max|ref| + 1e-2 * |ref|; sums relative 1e-5 (fp32 per-lane
partials, fp64 across blocks)."""
import importlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

PK_CONVT_FWD, PK_CONVT_DGRAD = 2, 3
REP = 16


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
    assert bad == 0, f"{bad} / {ref.numel()} elements off; max err {err.max().item():.4g}"


def pack(L, w, kind):
    Ci, Co = w.shape[:2]
    dst = torch.empty(w.numel(), dtype=torch.bfloat16, device="cuda")
    assert L.unet_pack_weight(w.data_ptr(), dst.data_ptr(), kind, Co, Ci, 2, 2, S()) == 0, L.unet_last_error()
    return dst


def convt(L, x, ldx, wp, y, ldy, N, H, W, Ci, Co, mode, grid=0, bias=None, bb=None, bias_acc=None):
    p = lambda t: 0 if t is None else t.data_ptr()
    bb = bb or {}
    act, yr = bb.get("act"), bb.get("y")
    rc = L.unet_convt2x2(p(x), ldx, p(wp), p(y), ldy, p(bias), p(act), 0 if act is None else act.shape[-1], p(yr),
                         0 if yr is None else yr.shape[-1], p(bb.get("mean")), p(bb.get("invstd")),
                         p(bb.get("sums")), p(bias_acc), N, H, W, Ci, Co, mode, grid, S())
    assert rc == 0, L.unet_last_error()


SHAPES = [(64, 32), (64, 64), (128, 64)]
GRIDS = [(2, 16, 24), (1, 32, 32), (3, 8, 16)]


@pytest.mark.parametrize("Ci,Co", SHAPES)
@pytest.mark.parametrize("N,H,W", GRIDS)
def test_convt_forward(L, Ci, Co, N, H, W, cuda):
    g = torch.Generator().manual_seed(5)
    x = bf(torch.randn(N, Ci, H, W, generator=g))
    w = torch.randn(Ci, Co, 2, 2, generator=g) / Ci ** 0.5
    b = torch.randn(Co, generator=g)
    ref = F.conv_transpose2d(x.float(), bf(w).float(), b, stride=2)
    wg, bg = w.cuda(), b.cuda()
    wp = pack(L, wg, PK_CONVT_FWD)
    xg = nhwc(x).cuda()
    off, ld = 32, Co + 48  # a concat slice: channels [off, off + Co) of an ld-channel buffer
    ybuf = torch.zeros(N, 2 * H, 2 * W, ld, dtype=torch.bfloat16, device="cuda")
    convt(L, xg, Ci, wp, ybuf[..., off:], ld, N, H, W, Ci, Co, 0, bias=bg)
    torch.cuda.synchronize()
    close(nchw(ybuf[..., off:off + Co]), ref)
    assert ybuf[..., :off].abs().sum().item() == 0 and ybuf[..., off + Co:].abs().sum().item() == 0
    # a capped grid walks more pixel groups per wave: same bits
    y2 = torch.zeros_like(ybuf)
    convt(L, xg, Ci, wp, y2[..., off:], ld, N, H, W, Ci, Co, 0, grid=3, bias=bg)
    torch.cuda.synchronize()
    assert torch.equal(y2, ybuf)


@pytest.mark.parametrize("Ci,Co", SHAPES)
@pytest.mark.parametrize("N,H,W", GRIDS)
@pytest.mark.parametrize("fused", [False, True])
def test_convt_dgrad(L, Ci, Co, N, H, W, fused, cuda):
    g = torch.Generator().manual_seed(6)
    w = torch.randn(Ci, Co, 2, 2, generator=g) / (4 * Co) ** 0.5
    dy = bf(torch.randn(N, Co, 2 * H, 2 * W, generator=g))
    xr = torch.zeros(N, Ci, H, W, requires_grad=True)
    F.conv_transpose2d(xr, bf(w).float(), None, stride=2).backward(dy.float())
    da = xr.grad  # dA wrt the up-conv input
    wp = pack(L, w.cuda(), PK_CONVT_DGRAD)
    off, ld = 64, Co + 64  # dY read from a concat slice, as decoder1's dcat
    dybuf = torch.zeros(N, 2 * H, 2 * W, ld, dtype=torch.bfloat16)
    dybuf[..., off:off + Co] = nhwc(dy)
    dybuf = dybuf.cuda()
    bb, act, yraw, mean, invstd = None, None, None, None, None
    if fused:
        act = bf(torch.randn(N, Ci, H, W, generator=g).clamp_min(0))  # ReLU output: ~half zeros
        yraw = bf(torch.randn(N, Ci, H, W, generator=g) * 2 + 0.5)
        mean = torch.randn(Ci, generator=g) * 0.3 + 0.5
        invstd = torch.rand(Ci, generator=g) + 0.5
        bb = {"act": nhwc(act).cuda(), "y": nhwc(yraw).cuda(), "mean": mean.cuda(), "invstd": invstd.cuda(),
              "sums": torch.zeros(REP * 2 * Ci, dtype=torch.float64, device="cuda")}
    bias_acc = torch.zeros(REP * Co, dtype=torch.float64, device="cuda")
    dx = torch.empty(N, H, W, Ci, dtype=torch.bfloat16, device="cuda")
    convt(L, dybuf[..., off:], ld, wp, dx, Ci, N, H, W, Ci, Co, 1, bb=bb, bias_acc=bias_acc)
    torch.cuda.synchronize()
    ref = da if not fused else da * (act.float() > 0)
    close(nchw(dx), ref)
    # bias gradient: the sum of dY over pixels and taps
    bsum = bias_acc.cpu().view(REP, Co).sum(0)
    torch.testing.assert_close(bsum, dy.double().sum((0, 2, 3)), rtol=1e-5, atol=1e-6 * dy.numel() ** 0.5)
    if fused:  # BN-backward sums of the STORED dZ (what bn_bwd_reduce_kernel would read back)
        dz = nchw(dx).double().cpu()
        xhat = (yraw.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
        s = bb["sums"].cpu().view(REP, 2, Ci).sum(0)
        scale = dz.abs().sum((0, 2, 3)).clamp_min(1e-30)
        assert ((s[0] - dz.sum((0, 2, 3))).abs() / scale).max().item() <= 1e-5
        assert ((s[1] - (dz * xhat).sum((0, 2, 3))).abs() / (dz * xhat).abs().sum((0, 2, 3)).clamp_min(1e-30)).max().item() <= 1e-5
    # capped grid: the stored dX / dZ are bit-identical
    dx2 = torch.empty_like(dx)
    bb2 = None if bb is None else dict(bb, sums=torch.zeros_like(bb["sums"]))
    convt(L, dybuf[..., off:], ld, wp, dx2, Ci, N, H, W, Ci, Co, 1, grid=2, bb=bb2,
          bias_acc=torch.zeros_like(bias_acc))
    torch.cuda.synchronize()
    assert torch.equal(dx2, dx)


def test_convt_rejects_uncovered(L, cuda):
    """(Ci, Co) outside the table and pixel counts not a multiple of 32 fail
    loudly (the executor falls back to the implicit GEMM for those)."""
    x = torch.zeros(1, 8, 8, 256, dtype=torch.bfloat16, device="cuda")
    wp = torch.zeros(256 * 128 * 4, dtype=torch.bfloat16, device="cuda")
    y = torch.zeros(1, 16, 16, 128, dtype=torch.bfloat16, device="cuda")
    assert L.unet_convt2x2(x.data_ptr(), 256, wp.data_ptr(), y.data_ptr(), 128, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                           1, 8, 8, 256, 128, 0, 0, S()) != 0
    x = torch.zeros(1, 3, 5, 64, dtype=torch.bfloat16, device="cuda")
    y = torch.zeros(1, 6, 10, 32, dtype=torch.bfloat16, device="cuda")
    assert L.unet_convt2x2(x.data_ptr(), 64, wp.data_ptr(), y.data_ptr(), 32, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                           1, 3, 5, 64, 32, 0, 0, S()) != 0
    torch.cuda.synchronize()
