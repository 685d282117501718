"""Local ("teacher-forced") parity of every op as the native executor composes
it: each forward/backward tensor in the workspace is recomputed in fp32 on the
CPU from the executor's OWN stored inputs (bf16) and compared.  Unlike an
end-to-end comparison this is immune to the depth-wise amplification of bf16
rounding in a randomly initialised BN network, so it pins the wiring (which
buffer feeds which op, skip/concat/residual gradient sums, bucket unpacking)
and each kernel at its true tolerance: relative L2 error <= 2e-2 per tensor.
"""
import os

import pytest
import torch
import torch.nn.functional as F

import oracle

pytestmark = pytest.mark.gpu
TOL = 2e-2


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def bn_train(v, mod, stats_from=None):
    s = v if stats_from is None else stats_from
    mean = s.mean((0, 2, 3), keepdim=True)
    var = s.var((0, 2, 3), unbiased=False, keepdim=True)
    return (v - mean) / torch.sqrt(var + 1e-5) * mod.weight.view(1, -1, 1, 1) + mod.bias.view(1, -1, 1, 1)


def local_bn_bwd(y, dout, mod, out=None, extra=None):
    """gradient wrt y (and extra leaves) of relu(bn(y) + extra_term)."""
    yl = y.clone().requires_grad_(True)
    g = mod.weight.detach().clone().requires_grad_(True)
    b = mod.bias.detach().clone().requires_grad_(True)
    z = F.batch_norm(yl, None, None, g, b, True, 0.1, 1e-5)
    leaves = [yl, g, b]
    if extra is not None:
        z = z + extra()
    o = F.relu(z)
    if out is not None:  # use the executor's stored relu mask
        o = z * (out > 0).float()
    o.backward(dout)
    return yl.grad, g.grad, b.grad


@pytest.fixture(scope="module", params=[(1, None), (2, None), (1, (1, 64, 96)), (1, (2, 256, 256)),
                                        (1, (1, 512, 512)), (1, (16, 256, 256))],
                ids=["base", "wide", "n1_64x96", "n2_256", "n1_512", "n16_256"])
def run(pkg, golden, cuda, request):
    """width 1 = Base topology; width 2 = the Wide config (every channel x2);
    n1_64x96 = a ragged case: batch 1, non-square, a 2x3 deepest level (the
    kernels' partial-tile and fallback paths); n2_256 = 256x256, large enough
    for the stride-2 halo weight gradients (enc2.0 / enc3.0 conv1 with the
    downsample's weight gradient folded in); n1_512 = one 512x512 image: the
    Base geometry, so enc4 (16 x 16) runs the 16-wide batched weight gradient;
    n16_256 = 16 images of 256x256: batch 16 wiring at a quarter of the bench's
    pixels.  Its enc2 / enc3 / decoder4 / decoder3 convs have 64-128 work items
    of 16 x 16 x 64, below the 256 CUs, so they run the halo-streamed kernel;
    only decoder2.0's forward (256 items) reaches the full-line kernel here.
    The full-line family (conv_fl.hip) is pinned at the bench's own 16 x 512^2
    workload in test_fl_routing_gpu.py (routing asserted per layer) and as a
    single op in test_conv_fl_gpu.py."""
    width, shape = request.param
    # the stem runs by recompute (stem_rc.hip) and stores neither its raw conv
    # output y0 nor the maxpool/BN dZ; keep both for the teacher-forced rows
    os.environ["UNET_STEM_KEEP"] = "1"
    base = golden("base64.npz")
    if shape is not None:
        xs, ms = pkg.synthetic_cells(*shape, seed=7)
        base = {"x": xs, "masks": ms}
    ref = oracle.ReferenceUNet(width=width)
    sd = oracle.closed_form_state_dict(ref, seed=0)
    ref.load_state_dict(sd)
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=False, width=width)
    m.load_state_dict(sd)
    m = m.cuda().train()
    x = torch.from_numpy(base["x"])
    y = torch.from_numpy(base["masks"])
    try:
        out = m(x.cuda())
        loss = pkg.get_loss_function({"loss_fn": "bce"})(out, y.cuda())
        loss.backward()
        torch.cuda.synchronize()
    finally:
        del os.environ["UNET_STEM_KEEP"]
    plan = m._last_plan
    v = {k: t.cpu() for k, t in plan.tensor_views().items()}
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters()}
    return ref, x, y, out.detach().cpu(), v, grads


def _masked(a, b, act):
    """dA buffers consumed by a BN+ReLU hold dZ = dA * (act > 0) when the BN
    backward reduction is fused into their producer: compare under the mask."""
    m = (act > 0).float()
    return _rel(a * m, b * m)


def _dcat(v, p):
    """concat gradient of decoder p: one buffer, or (decoder1) the skip part and
    the narrow up-conv part the executor keeps in separate dense buffers."""
    if p + "d.cat" in v:
        return v[p + "d.cat"]
    return torch.cat([v[p + "d.cat.skip"], v[p + "d.cat.up"]], 1)


def dec1_act(v, bn):
    """decoder1's output act = relu(bn2(y2)) in bf16.  A training forward does
    not store it (HeadArgs.bn_fold: the head applies that BN + ReLU to y2 in
    both of its passes), so the head rows are teacher-forced from y2; the
    logits / dA / upconv0 / conv_final rows then check the fold itself."""
    with torch.no_grad():
        return F.relu(bn_train(v["dec1.y2"], bn)).to(torch.bfloat16).float()


def _check(rows):
    for name, e in rows:
        print(f"{name:28s} {e:.3e}")
    bad = [(n, e) for n, e in rows if not e <= TOL]
    assert not bad, bad


def test_forward_ops(run):
    ref, x, y, logits, v, _ = run
    W = lambda mod: mod.weight.detach().to(torch.bfloat16).float()
    rows = []
    with torch.no_grad():
        xq = x.to(torch.bfloat16).float()
        y0f = F.conv2d(xq, W(ref.input_conv), stride=2, padding=3)
        rows.append(("y0", _rel(v["y0"], y0f)))
        # the stem normalises its fp32 conv output (stem_rc.hip), not the bf16 y0 kept for tests
        rows.append(("x1", _rel(v["x1"], F.relu(bn_train(y0f, ref.bn1)))))
        rows.append(("p0", _rel(v["p0"], F.max_pool2d(v["x1"], 3, 2, 1))))
        prev = v["p0"]
        for s, stage in enumerate((ref.enc1, ref.enc2, ref.enc3, ref.enc4)):
            for b, blk in enumerate(stage):
                p = f"enc{s + 1}.{b}."
                st = blk.conv1.stride
                rows.append((p + "y1", _rel(v[p + "y1"], F.conv2d(prev, W(blk.conv1), stride=st, padding=1))))
                rows.append((p + "h", _rel(v[p + "h"], F.relu(bn_train(v[p + "y1"], blk.bn1)))))
                rows.append((p + "y2", _rel(v[p + "y2"], F.conv2d(v[p + "h"], W(blk.conv2), padding=1))))
                if blk.downsample is not None:
                    rows.append((p + "yds", _rel(v[p + "yds"], F.conv2d(prev, W(blk.downsample[0]), stride=st))))
                    skip = bn_train(v[p + "yds"], blk.downsample[1])
                else:
                    skip = prev
                rows.append((p + "out", _rel(v[p + "out"], F.relu(bn_train(v[p + "y2"], blk.bn2) + skip))))
                prev = v[p + "out"]
        skips = {4: v["enc3.5.out"], 3: v["enc2.3.out"], 2: v["enc1.2.out"], 1: v["x1"]}
        for lvl in (4, 3, 2, 1):
            up, dec, p = getattr(ref, f"upconv{lvl}"), getattr(ref, f"decoder{lvl}"), f"dec{lvl}."
            rows.append((p + "up", _rel(v[p + "up"], F.conv_transpose2d(prev, W(up), up.bias, stride=2))))
            rows.append((p + "cat", _rel(v[p + "cat"], torch.cat((skips[lvl], v[p + "up"]), 1))))
            rows.append((p + "y1", _rel(v[p + "y1"], F.conv2d(v[p + "cat"], W(dec[0]), dec[0].bias, padding=1))))
            rows.append((p + "h", _rel(v[p + "h"], F.relu(bn_train(v[p + "y1"], dec[1])))))
            rows.append((p + "y2", _rel(v[p + "y2"], F.conv2d(v[p + "h"], W(dec[3]), dec[3].bias, padding=1))))
            if lvl == 1:
                break  # decoder1's act is formed inside the head (dec1_act)
            rows.append((p + "out", _rel(v[p + "out"], F.relu(bn_train(v[p + "y2"], dec[4])))))
            prev = v[p + "out"]
        head = ref.conv_final(ref.upconv0(dec1_act(v, ref.decoder1[4])))
        rows.append(("logits", _rel(logits, head)))
    _check(rows)


def test_backward_ops(run):
    ref, x, y, logits, v, grads = run
    W = lambda mod: mod.weight.detach().to(torch.bfloat16).float()
    rows = []
    n = logits.numel()
    dl = (torch.sigmoid(logits) - y) / n
    # head: upconv0 + conv_final
    a1 = dec1_act(v, ref.decoder1[4])
    d1 = a1.clone().requires_grad_(True)
    u0w = ref.upconv0.weight.detach().clone().requires_grad_(True)
    u0b = ref.upconv0.bias.detach().clone().requires_grad_(True)
    fw = ref.conv_final.weight.detach().clone().requires_grad_(True)
    fb = ref.conv_final.bias.detach().clone().requires_grad_(True)
    F.conv2d(F.conv_transpose2d(d1, u0w, u0b, stride=2), fw, fb).backward(dl)
    rows += [("dec1.d.out", _masked(v["dec1.d.out"], d1.grad, a1)), ("g upconv0.weight", _rel(grads["upconv0.weight"], u0w.grad)),
             ("g upconv0.bias", _rel(grads["upconv0.bias"], u0b.grad)),
             ("g conv_final.weight", _rel(grads["conv_final.weight"], fw.grad)),
             ("g conv_final.bias", _rel(grads["conv_final.bias"], fb.grad))]
    dprev = None
    skips = {4: ("enc3.5.out", 256), 3: ("enc2.3.out", 128), 2: ("enc1.2.out", 64), 1: ("x1", 64)}
    for lvl in (1, 2, 3, 4):
        dec, up, p = getattr(ref, f"decoder{lvl}"), getattr(ref, f"upconv{lvl}"), f"dec{lvl}."
        dout = v[p + "d.out"]
        dy2, dg, db = local_bn_bwd(v[p + "y2"], dout, dec[4], out=a1 if lvl == 1 else v[p + "out"])
        rows += [(p + "d.y2", _rel(v[p + "d.y2"], dy2)), (f"g decoder{lvl}.4.weight", _rel(grads[f"decoder{lvl}.4.weight"], dg)),
                 (f"g decoder{lvl}.4.bias", _rel(grads[f"decoder{lvl}.4.bias"], db))]
        dh = torch.nn.grad.conv2d_input(v[p + "h"].shape, W(dec[3]), v[p + "d.y2"], padding=1)
        rows.append((p + "d.h", _masked(v[p + "d.h"], dh, v[p + "h"])))
        gw = torch.nn.grad.conv2d_weight(v[p + "h"], dec[3].weight.shape, v[p + "d.y2"], padding=1)
        rows.append((f"g decoder{lvl}.3.weight", _rel(grads[f"decoder{lvl}.3.weight"], gw)))
        dy1, dg, db = local_bn_bwd(v[p + "y1"], v[p + "d.h"], dec[1], out=v[p + "h"])
        rows += [(p + "d.y1", _rel(v[p + "d.y1"], dy1)), (f"g decoder{lvl}.1.weight", _rel(grads[f"decoder{lvl}.1.weight"], dg))]
        dcat = torch.nn.grad.conv2d_input(v[p + "cat"].shape, W(dec[0]), v[p + "d.y1"], padding=1)
        rows.append((p + "d.cat", _rel(_dcat(v, p), dcat)))
        gw = torch.nn.grad.conv2d_weight(v[p + "cat"], dec[0].weight.shape, v[p + "d.y1"], padding=1)
        rows.append((f"g decoder{lvl}.0.weight", _rel(grads[f"decoder{lvl}.0.weight"], gw)))
        sk = v[skips[lvl][0]].shape[1]
        du = _dcat(v, p)[:, sk:]
        upin_name = "enc4.2.out" if lvl == 4 else f"dec{lvl + 1}.out"
        xin = v[upin_name].clone().requires_grad_(True)
        wl = W(up).clone().requires_grad_(True)
        bl = up.bias.detach().clone().requires_grad_(True)
        F.conv_transpose2d(xin, wl, bl, stride=2).backward(du)
        tgt = "enc4.2.d.out" if lvl == 4 else f"dec{lvl + 1}.d.out"
        rows += [(tgt + " (convT dgrad)", _masked(v[tgt], xin.grad, v[upin_name])),
                 (f"g upconv{lvl}.weight", _rel(grads[f"upconv{lvl}.weight"], wl.grad)),
                 (f"g upconv{lvl}.bias", _rel(grads[f"upconv{lvl}.bias"], bl.grad))]
    # encoder blocks
    names = []
    for s, stage in enumerate((ref.enc1, ref.enc2, ref.enc3, ref.enc4)):
        for b, blk in enumerate(stage):
            names.append((f"enc{s + 1}.{b}.", blk, s, b))
    for i in range(len(names) - 1, -1, -1):
        p, blk, s, b = names[i]
        inp = v["p0"] if i == 0 else v[names[i - 1][0] + "out"]
        dout = v[p + "d.out"]
        y2 = v[p + "y2"].clone().requires_grad_(True)
        g2 = blk.bn2.weight.detach().clone().requires_grad_(True)
        b2 = blk.bn2.bias.detach().clone().requires_grad_(True)
        z = F.batch_norm(y2, None, None, g2, b2, True, 0.1, 1e-5)
        if blk.downsample is not None:
            yds = v[p + "yds"].clone().requires_grad_(True)
            gd = blk.downsample[1].weight.detach().clone().requires_grad_(True)
            bd = blk.downsample[1].bias.detach().clone().requires_grad_(True)
            z = z + F.batch_norm(yds, None, None, gd, bd, True, 0.1, 1e-5)
            skip = None
        else:
            skip = inp.clone().requires_grad_(True)
            z = z + skip
        (z * (v[p + "out"] > 0).float()).backward(dout)
        rows += [(p + "d.y2", _rel(v[p + "d.y2"], y2.grad)), (f"g {p}bn2.weight", _rel(grads[p + "bn2.weight"], g2.grad)),
                 (f"g {p}bn2.bias", _rel(grads[p + "bn2.bias"], b2.grad))]
        if blk.downsample is not None:
            rows += [(p + "d.yds", _rel(v[p + "d.yds"], yds.grad)),
                     (f"g {p}downsample.1.weight", _rel(grads[p + "downsample.1.weight"], gd.grad)),
                     (f"g {p}downsample.1.bias", _rel(grads[p + "downsample.1.bias"], bd.grad))]
        dh = torch.nn.grad.conv2d_input(v[p + "h"].shape, W(blk.conv2), v[p + "d.y2"], padding=1)
        rows.append((p + "d.h", _masked(v[p + "d.h"], dh, v[p + "h"])))
        rows.append((f"g {p}conv2.weight", _rel(grads[p + "conv2.weight"],
                                                 torch.nn.grad.conv2d_weight(v[p + "h"], blk.conv2.weight.shape, v[p + "d.y2"], padding=1))))
        dy1, dg, db = local_bn_bwd(v[p + "y1"], v[p + "d.h"], blk.bn1, out=v[p + "h"])
        rows += [(p + "d.y1", _rel(v[p + "d.y1"], dy1)), (f"g {p}bn1.weight", _rel(grads[p + "bn1.weight"], dg))]
        st = blk.conv1.stride
        din = torch.nn.grad.conv2d_input(inp.shape, W(blk.conv1), v[p + "d.y1"], stride=st, padding=1)
        if blk.downsample is not None:
            din = din + torch.nn.grad.conv2d_input(inp.shape, W(blk.downsample[0]), v[p + "d.yds"], stride=st)
            rows.append((f"g {p}downsample.0.weight", _rel(grads[p + "downsample.0.weight"], torch.nn.grad.conv2d_weight(
                inp, blk.downsample[0].weight.shape, v[p + "d.yds"], stride=st))))
        else:
            din = din + skip.grad
        if b == 0 and s > 0:
            lvl = {1: 2, 2: 3, 3: 4}[s]
            din = din + _dcat(v, f"dec{lvl}.")[:, :inp.shape[1]]
        tgt = "d.p0" if i == 0 else names[i - 1][0] + "d.out"
        rows.append((tgt + " (block dgrad)", _rel(v[tgt], din) if i == 0 else _masked(v[tgt], din, inp)))
        rows.append((f"g {p}conv1.weight", _rel(grads[p + "conv1.weight"], torch.nn.grad.conv2d_weight(
            inp, blk.conv1.weight.shape, v[p + "d.y1"], stride=st, padding=1))))
    # maxpool + stem
    x1 = v["x1"].clone().requires_grad_(True)
    F.max_pool2d(x1, 3, 2, 1).backward(v["d.p0"])
    rows.append(("d.x1", _masked(v["d.x1"], x1.grad + _dcat(v, "dec1.")[:, :v["x1"].shape[1]], v["x1"])))
    xq = x.to(torch.bfloat16).float()
    y0f = F.conv2d(xq, W(ref.input_conv), stride=2, padding=3)  # fp32, as the stem normalises it
    dy0, dg, db = local_bn_bwd(y0f, v["d.x1"], ref.bn1, out=v["x1"])
    rows += [("g bn1.weight", _rel(grads["bn1.weight"], dg)), ("g bn1.bias", _rel(grads["bn1.bias"], db))]
    if "d.y0" in v:  # unfused build only: the fused stem wgrad never stores the stem dY
        rows.append(("d.y0", _rel(v["d.y0"], dy0)))
    rows.append(("g input_conv.weight", _rel(grads["input_conv.weight"], torch.nn.grad.conv2d_weight(
        xq, ref.input_conv.weight.shape, dy0, stride=2, padding=3))))
    _check(rows)
