"""The full-line halo conv family (conv3x3_fl_kernel, conv_fl.hip) at the
bench's own workload -- BASELINE.json configs[1], Base U-Net 16 x 512^2 --
VERDICT r05 item 1.

1. Routing: one training step with the per-launch profiler on; every launch
   whose kernel is a conv3x3_fl_kernel instance is listed with its template
   tag and compared with the expected table below (which layer, forward or
   data gradient, which epilogue instance).  A gate change (e.g. the CU-count
   fill rule of conv3x3_fl_shape) or an epilogue change fails here instead of
   silently routing a layer to the halo-streamed kernel.
2. Teacher-forced parity of every fl layer in that same step: each output the
   kernel writes is recomputed in fp32 on the CPU from the executor's OWN bf16
   inputs (as test_wiring_gpu.py), and so is every quantity the fused epilogues
   feed: the BN-backward results that consume the fused (sum dZ, sum dZ*xhat)
   sums -- the bn1 / bn2 / downsample BN gradients and dY of the next apply --
   and, for the two-BN <true, true, 32> instance, both BNs.  Bar: relative L2
   <= 2e-2 per tensor (measured ~2e-3 at smaller sizes).

Covered instances (16 x 512^2, 256 CUs): forward <false, false, 8> (23
launches: enc2 / enc3 3x3 convs, decoder4 / decoder3, decoder2.0; enc2 has 2
work items per block, so the persistent multi-item path runs); data gradient
<true, false, 12> (fused BN backward), <true, false, 14> (+ residual addend),
<true, false, 0> (decoder4.0 / decoder3.0: the concat gradient, no BN) and
<true, true, 32> (enc2.1 / enc3.1 conv1: the downsample block's two BNs).
Reference: /root/reference/advanced_models.py:84-87 (BasicBlock), :197-205
(decoder blocks)."""
import pytest
import torch
import torch.nn.functional as F

import oracle

pytestmark = pytest.mark.gpu
TOL = 2e-2
N_IMG, SIZE = 16, 512

FWD8 = "conv3x3_fl_kernel<false, false, 8>"
D12, D14, D0, TWO = ("conv3x3_fl_kernel<true, false, 12>", "conv3x3_fl_kernel<true, false, 14>",
                     "conv3x3_fl_kernel<true, false, 0>", "conv3x3_fl_kernel<true, true, 32>")


def expected_routing():
    """{launch name: kernel tag} of every fl launch of one Base 16 x 512^2 step
    on a 256-CU MI355X (profiles/r05/s5/layer_profile.txt lists the same)."""
    e = {}
    for s, nb in ((2, 4), (3, 6)):
        for b in range(nb):
            p = f"enc{s}.{b}."
            e[f"fwd {p}conv2.weight"] = FWD8
            e[f"dgrad {p}conv2.weight"] = D12          # produces dA of bn1: fused BN backward
            if b > 0:
                e[f"fwd {p}conv1.weight"] = FWD8
                # dA of the previous block's output: identity residual (+addend),
                # or the downsample block's two BNs (b == 1)
                e[f"dgrad {p}conv1.weight"] = TWO if b == 1 else D14
    for lvl in (4, 3):
        e[f"fwd decoder{lvl}.0.weight"] = FWD8
        e[f"fwd decoder{lvl}.3.weight"] = FWD8
        e[f"dgrad decoder{lvl}.0.weight"] = D0         # the concat gradient (no BN)
        e[f"dgrad decoder{lvl}.3.weight"] = D12
    e["fwd decoder2.0.weight"] = FWD8
    return e


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _masked(a, b, act):
    m = (act > 0).float()
    return _rel(a * m, b * m)


@pytest.fixture(scope="module")
def step(pkg, cuda):
    ref = oracle.ReferenceUNet()
    sd = oracle.closed_form_state_dict(ref, seed=0)
    ref.load_state_dict(sd)
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=False)
    m.load_state_dict(sd)
    m = m.cuda().train()
    xs, ms = pkg.synthetic_cells(N_IMG, SIZE, SIZE, seed=7)
    x, y = torch.from_numpy(xs).cuda(), torch.from_numpy(ms).cuda()
    crit = pkg.get_loss_function({"loss_fn": "bce"})

    def one_step():
        m.zero_grad(set_to_none=False)
        crit(m(x), y).backward()

    one_step()  # creates the plan
    plan = m._last_plan
    plan.profile(True)
    one_step()
    torch.cuda.synchronize()
    recs = plan.profile_report()
    plan.profile(False)
    v = {k: t.cpu() for k, t in plan.tensor_views().items()}
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters()}
    return ref, recs, v, grads


def test_fl_routing_matches_table(step):
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if ncu != 256:
        pytest.skip(f"routing table is for 256 CUs (this device has {ncu})")
    _, recs, _, _ = step
    got = {name: kern for name, _, _, kern in recs if kern.startswith("conv3x3_fl_kernel")}
    exp = expected_routing()
    missing = {k: v for k, v in exp.items() if k not in got}
    extra = {k: v for k, v in got.items() if k not in exp}
    wrong = {k: (got[k], v) for k, v in exp.items() if k in got and got[k] != v}
    assert not missing and not extra and not wrong, (missing, extra, wrong)
    assert len(got) == 45 and sum(1 for t in got.values() if t == FWD8) == 23
    # every instance family of the bench is reached
    assert set(got.values()) == {FWD8, D12, D14, D0, TWO}


def bn_train(v, mod):
    mean = v.mean((0, 2, 3), keepdim=True)
    var = v.var((0, 2, 3), unbiased=False, keepdim=True)
    return (v - mean) / torch.sqrt(var + 1e-5) * mod.weight.view(1, -1, 1, 1) + mod.bias.view(1, -1, 1, 1)


def _check(rows):
    for name, e in rows:
        print(f"{name:40s} {e:.3e}")
    bad = [(n, e) for n, e in rows if not e <= TOL]
    assert not bad, bad


def test_fl_forward_teacher_forced(step):
    ref, _, v, _ = step
    W = lambda mod: mod.weight.detach().to(torch.bfloat16).float()
    rows = []
    with torch.no_grad():
        for s, stage in ((2, ref.enc2), (3, ref.enc3)):
            for b, blk in enumerate(stage):
                p = f"enc{s}.{b}."
                prev = v[f"enc{s}.{b - 1}.out"] if b > 0 else None
                if b > 0:
                    rows.append((p + "y1", _rel(v[p + "y1"], F.conv2d(prev.float(), W(blk.conv1), padding=1))))
                rows.append((p + "y2", _rel(v[p + "y2"], F.conv2d(v[p + "h"].float(), W(blk.conv2), padding=1))))
        for lvl in (4, 3, 2):
            dec, p = getattr(ref, f"decoder{lvl}"), f"dec{lvl}."
            rows.append((p + "y1", _rel(v[p + "y1"], F.conv2d(v[p + "cat"].float(), W(dec[0]), dec[0].bias,
                                                               padding=1))))
            if lvl != 2:
                rows.append((p + "y2", _rel(v[p + "y2"], F.conv2d(v[p + "h"].float(), W(dec[3]), dec[3].bias,
                                                                   padding=1))))
    _check(rows)


def _bn_relu_bwd(y, dout, mod, out, extra=None):
    """d/dy (and gamma / beta) of relu(bn(y) [+ extra]) under the executor's
    stored ReLU mask `out`; extra: (y2, mod2) of a second BN (downsample)."""
    yl = y.float().clone().requires_grad_(True)
    g = mod.weight.detach().clone().requires_grad_(True)
    b = mod.bias.detach().clone().requires_grad_(True)
    z = F.batch_norm(yl, None, None, g, b, True, 0.1, 1e-5)
    leaves = [yl, g, b]
    if extra is not None:
        y2, mod2 = extra
        y2l = y2.float().clone().requires_grad_(True)
        g2 = mod2.weight.detach().clone().requires_grad_(True)
        b2 = mod2.bias.detach().clone().requires_grad_(True)
        z = z + F.batch_norm(y2l, None, None, g2, b2, True, 0.1, 1e-5)
        leaves += [y2l, g2, b2]
    (z * (out > 0).float()).backward(dout.float())
    return [t.grad for t in leaves]


def test_fl_dgrad_teacher_forced(step):
    """Every fl data gradient and what its fused epilogue feeds."""
    ref, _, v, grads = step
    W = lambda mod: mod.weight.detach().to(torch.bfloat16).float()
    cin = torch.nn.grad.conv2d_input
    rows = []
    # encoder blocks: conv2 dgrad (<true,false,12>) -> d.h (dZ of bn1) and its BN backward
    for s, stage in ((2, ref.enc2), (3, ref.enc3)):
        for b, blk in enumerate(stage):
            p = f"enc{s}.{b}."
            dh = cin(v[p + "h"].shape, W(blk.conv2), v[p + "d.y2"].float(), padding=1)
            rows.append((p + "d.h  [conv2 dgrad]", _masked(v[p + "d.h"].float(), dh, v[p + "h"])))
            dy1, dg, db = _bn_relu_bwd(v[p + "y1"], v[p + "d.h"], blk.bn1, v[p + "h"])
            rows += [(p + "d.y1 [fused bn1 sums]", _rel(v[p + "d.y1"], dy1)),
                     (f"g {p}bn1.weight", _rel(grads[p + "bn1.weight"], dg)),
                     (f"g {p}bn1.bias", _rel(grads[p + "bn1.bias"], db))]
            if b == 0:
                continue
            # conv1 dgrad of block b >= 1 -> dA of block b-1's output (+ the residual dZ of block b)
            q = f"enc{s}.{b - 1}."
            prv = stage[b - 1]
            din = cin(v[q + "out"].shape, W(blk.conv1), v[p + "d.y1"].float(), padding=1)
            din = din + v[p + "d.out"].float() * (v[p + "out"] > 0).float()   # identity skip: dZ of block b
            tag = "TWO" if b == 1 else "14"
            rows.append((q + f"d.out [conv1 dgrad <{tag}>]", _masked(v[q + "d.out"].float(), din, v[q + "out"])))
            # the BN backward fed by the fused sums: bn2 (and the downsample BN for b == 1)
            if prv.downsample is not None:
                dy2, dg, db, dyds, dgd, dbd = _bn_relu_bwd(v[q + "y2"], v[q + "d.out"], prv.bn2, v[q + "out"],
                                                           extra=(v[q + "yds"], prv.downsample[1]))
                rows += [(q + "d.yds [two-BN sums]", _rel(v[q + "d.yds"], dyds)),
                         (f"g {q}downsample.1.weight", _rel(grads[q + "downsample.1.weight"], dgd)),
                         (f"g {q}downsample.1.bias", _rel(grads[q + "downsample.1.bias"], dbd))]
            else:
                dy2, dg, db = _bn_relu_bwd(v[q + "y2"], v[q + "d.out"], prv.bn2, v[q + "out"])
            rows += [(q + "d.y2 [fused bn2 sums]", _rel(v[q + "d.y2"], dy2)),
                     (f"g {q}bn2.weight", _rel(grads[q + "bn2.weight"], dg)),
                     (f"g {q}bn2.bias", _rel(grads[q + "bn2.bias"], db))]
    # decoders 4 / 3: dec.3 dgrad (<true,false,12>) -> d.h + dec.1 BN backward; dec.0 dgrad (<true,false,0>) -> d.cat
    for lvl in (4, 3):
        dec, p = getattr(ref, f"decoder{lvl}"), f"dec{lvl}."
        dh = cin(v[p + "h"].shape, W(dec[3]), v[p + "d.y2"].float(), padding=1)
        rows.append((p + "d.h  [dec.3 dgrad]", _masked(v[p + "d.h"].float(), dh, v[p + "h"])))
        dy1, dg, db = _bn_relu_bwd(v[p + "y1"], v[p + "d.h"], dec[1], v[p + "h"])
        rows += [(p + "d.y1 [fused dec.1 sums]", _rel(v[p + "d.y1"], dy1)),
                 (f"g decoder{lvl}.1.weight", _rel(grads[f"decoder{lvl}.1.weight"], dg)),
                 (f"g decoder{lvl}.1.bias", _rel(grads[f"decoder{lvl}.1.bias"], db))]
        dcat = cin(v[p + "cat"].shape, W(dec[0]), v[p + "d.y1"].float(), padding=1)
        rows.append((p + "d.cat [dec.0 dgrad <0>]", _rel(v[p + "d.cat"].float(), dcat)))
    _check(rows)
