"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the survey container (it reads /root/reference, which does not
exist on the GPU box).  It imports the reference's own ``advanced_models``,
``losses``, ``utils`` and ``train`` modules.  torchvision, cv2 and albumentations
are absent here, so three offline stand-in modules are written to a temp dir
first:

* ``torchvision.models.resnet34/resnet50(weights=None)`` rebuilt from
  torchvision's published ResNet layout (conv1/bn1/relu/maxpool/layer1-4,
  BasicBlock conv1/bn1/conv2/bn2/downsample.{0,1});
* empty ``cv2`` and ``albumentations`` modules (the hot path never calls them).

It then checks that ``oracle/`` is ``torch.equal`` to the reference on every
fixture and writes the vectors.  Nothing from the reference is copied: only
inputs and outputs are stored.

Usage:  python tests/golden/make_golden.py [--only-r50]
"""
from __future__ import annotations

import importlib.util
import os
import sys
import tempfile
import textwrap

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

TV_STANDIN = textwrap.dedent('''
    import torch.nn as nn

    def _c3(i, o, s=1):
        return nn.Conv2d(i, o, 3, s, 1, bias=False)

    class BasicBlock(nn.Module):
        expansion = 1
        def __init__(self, inplanes, planes, stride=1, downsample=None):
            super().__init__()
            self.conv1 = _c3(inplanes, planes, stride)
            self.bn1 = nn.BatchNorm2d(planes)
            self.relu = nn.ReLU(inplace=True)
            self.conv2 = _c3(planes, planes)
            self.bn2 = nn.BatchNorm2d(planes)
            self.downsample = downsample
            self.stride = stride
        def forward(self, x):
            idt = x
            out = self.relu(self.bn1(self.conv1(x)))
            out = self.bn2(self.conv2(out))
            if self.downsample is not None:
                idt = self.downsample(x)
            out += idt
            return self.relu(out)

    class Bottleneck(nn.Module):
        expansion = 4
        def __init__(self, inplanes, planes, stride=1, downsample=None):
            super().__init__()
            self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
            self.bn1 = nn.BatchNorm2d(planes)
            self.conv2 = _c3(planes, planes, stride)
            self.bn2 = nn.BatchNorm2d(planes)
            self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
            self.bn3 = nn.BatchNorm2d(planes * 4)
            self.relu = nn.ReLU(inplace=True)
            self.downsample = downsample
            self.stride = stride
        def forward(self, x):
            idt = x
            out = self.relu(self.bn1(self.conv1(x)))
            out = self.relu(self.bn2(self.conv2(out)))
            out = self.bn3(self.conv3(out))
            if self.downsample is not None:
                idt = self.downsample(x)
            out += idt
            return self.relu(out)

    class ResNet(nn.Module):
        def __init__(self, block, layers):
            super().__init__()
            self.inplanes = 64
            self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
            self.bn1 = nn.BatchNorm2d(64)
            self.relu = nn.ReLU(inplace=True)
            self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
            self.layer1 = self._make(block, 64, layers[0])
            self.layer2 = self._make(block, 128, layers[1], 2)
            self.layer3 = self._make(block, 256, layers[2], 2)
            self.layer4 = self._make(block, 512, layers[3], 2)
            self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
            self.fc = nn.Linear(512 * block.expansion, 1000)
        def _make(self, block, planes, blocks, stride=1):
            ds = None
            if stride != 1 or self.inplanes != planes * block.expansion:
                ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                   nn.BatchNorm2d(planes * block.expansion))
            layers = [block(self.inplanes, planes, stride, ds)]
            self.inplanes = planes * block.expansion
            layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
            return nn.Sequential(*layers)

    def resnet34(weights=None, **kw):
        assert weights is None, "offline stand-in: no pretrained weights"
        return ResNet(BasicBlock, [3, 4, 6, 3])

    def resnet50(weights=None, **kw):
        assert weights is None, "offline stand-in: no pretrained weights"
        return ResNet(Bottleneck, [3, 4, 6, 3])

    def densenet121(weights=None, **kw):
        raise NotImplementedError("densenet121 stand-in not provided")
''')


def _import_reference():
    tmp = tempfile.mkdtemp(prefix="refshim_")
    os.makedirs(os.path.join(tmp, "torchvision", "models"))
    with open(os.path.join(tmp, "torchvision", "__init__.py"), "w") as f:
        f.write("from . import models\n")
    with open(os.path.join(tmp, "torchvision", "models", "__init__.py"), "w") as f:
        f.write(TV_STANDIN)
    for name in ("cv2", "albumentations"):
        with open(os.path.join(tmp, name + ".py"), "w") as f:
            f.write("# offline stand-in: never called on the training hot path\n")
    sys.path.insert(0, tmp)
    sys.path.insert(0, REF)
    import advanced_models, losses, utils, train  # noqa: E401
    return advanced_models, losses, utils, train


def _load_synthetic():
    path = os.path.join(REPO, "image-segmentation-project_amd", "synthetic.py")
    spec = importlib.util.spec_from_file_location("_synthetic", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _proj(t: torch.Tensor, stream: int) -> float:
    from oracle import hash_uniform
    v = torch.from_numpy(hash_uniform(stream, t.numel())).to(torch.float64)
    return float((t.detach().double().reshape(-1) * v).sum())


def resnet50_fixture(am, ref_losses, oracle, syn):
    """backbone='resnet50' (advanced_models.py:102-130): the Bottleneck encoder
    and its decoder, with and without attention, at 2x1x64x64."""
    x_np, m_np = syn.synthetic_cells(2, 64, 64, seed=4321)
    x, m = torch.from_numpy(x_np), torch.from_numpy(m_np)
    out = {"x": x_np, "masks": m_np}
    for att in (False, True):
        tag = "att_" if att else ""
        torch.manual_seed(0)
        ref = am.UNetWithBackbone(n_classes=1, backbone="resnet50", pretrained=False, use_attention=att)
        orc = oracle.ReferenceUNet(backbone="resnet50", use_attention=att)
        rk = [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
        ok = [(k, tuple(v.shape)) for k, v in orc.state_dict().items()]
        assert rk == ok, "resnet50 state_dict layout differs from the reference"
        sd = oracle.closed_form_state_dict(orc, seed=0)
        ref.load_state_dict(sd); orc.load_state_dict(sd)
        ref.train(); orc.train()
        lr_ = ref(x); lo_ = orc(x)
        assert torch.equal(lr_, lo_), "resnet50: oracle logits != reference logits"
        loss_r = ref_losses.get_loss_function({"loss_fn": "bce"})(lr_, m)
        loss_o = oracle.get_loss_function({"loss_fn": "bce"})(lo_, m)
        assert torch.equal(loss_r, loss_o)
        loss_r.backward(); loss_o.backward()
        gr = dict(ref.named_parameters()); go = dict(orc.named_parameters())
        for k in gr:
            assert torch.equal(gr[k].grad, go[k].grad), k
        out[tag + "n_params"] = np.int64(sum(p.numel() for p in ref.parameters()))
        out[tag + "logits_train"] = lr_.detach().numpy()
        out[tag + "loss_bce"] = np.float32(loss_r.item())
        for k in ("conv_final.weight", "conv_final.bias", "upconv0.weight", "enc4.2.bn3.weight"):
            out[tag + "grad/" + k] = gr[k].grad.numpy().copy()
        bref = dict(ref.named_buffers())
        for k in ("bn1.running_mean", "enc1.0.bn3.running_var", "enc4.2.bn3.running_mean"):
            out[tag + "buf/" + k] = bref[k].numpy().copy()
        ref.load_state_dict(sd); orc.load_state_dict(sd)
        ref.eval(); orc.eval()
        with torch.no_grad():
            le = ref(x); lo = orc(x)
        assert torch.equal(le, lo)
        out[tag + "logits_eval"] = le.numpy()
    np.savez_compressed(os.path.join(HERE, "r50_64.npz"), **out)
    print("r50_64.npz: params", int(out["n_params"]), int(out["att_n_params"]), "bce", out["loss_bce"])


def main():
    sys.path.insert(0, REPO)
    torch.set_num_threads(8)
    am, ref_losses, ref_utils, ref_train = _import_reference()
    import oracle
    syn = _load_synthetic()
    if "--only-r50" in sys.argv:
        resnet50_fixture(am, ref_losses, oracle, syn)
        return

    # ---------------- base topology at 4x1x64x64 ----------------
    torch.manual_seed(0)
    ref = am.UNetWithBackbone(n_classes=1, backbone="resnet34", pretrained=False, use_attention=False)
    orc = oracle.ReferenceUNet()
    rk = [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
    ok = [(k, tuple(v.shape)) for k, v in orc.state_dict().items()]
    assert rk == ok, "state_dict layout differs from the reference"
    sd = oracle.closed_form_state_dict(orc, seed=0)
    ref.load_state_dict(sd)
    orc.load_state_dict(sd)
    n_params = sum(p.numel() for p in ref.parameters())

    x_np, m_np = syn.synthetic_cells(4, 64, 64, seed=1234)
    x, m = torch.from_numpy(x_np), torch.from_numpy(m_np)

    out = {"x": x_np, "masks": m_np, "n_params": np.int64(n_params)}
    names = [k for k, _ in ref.named_parameters()]
    bufnames = [k for k, _ in ref.named_buffers()]

    # train-mode forward + bce backward + one Adam step, reference path
    ref.train(); orc.train()
    crit_ref = ref_losses.get_loss_function({"loss_fn": "bce"})
    crit_orc = oracle.get_loss_function({"loss_fn": "bce"})
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
    opt_orc = oracle.make_adam(orc)
    lr_ = ref(x); lo_ = orc(x)
    assert torch.equal(lr_, lo_), "oracle logits != reference logits"
    loss_r = crit_ref(lr_, m); loss_o = crit_orc(lo_, m)
    assert torch.equal(loss_r, loss_o)
    for cfg in ({"loss_fn": "dice"}, {"loss_fn": "combo"}, {"loss_fn": "bogus"}):
        a = ref_losses.get_loss_function(cfg)(lr_, m)
        b = oracle.get_loss_function(cfg)(lo_, m)
        assert torch.equal(a, b), cfg
        out["loss_" + cfg["loss_fn"]] = np.float32(a.item())
    opt_ref.zero_grad(); loss_r.backward()
    opt_orc.zero_grad(); loss_o.backward()
    gr = dict(ref.named_parameters()); go = dict(orc.named_parameters())
    for k in names:
        assert torch.equal(gr[k].grad, go[k].grad), k
    out["logits_train"] = lr_.detach().numpy()
    out["loss_bce"] = np.float32(loss_r.item())
    out["grad_sumsq"] = np.array([float(gr[k].grad.double().pow(2).sum()) for k in names])
    out["grad_proj"] = np.array([_proj(gr[k].grad, 7000 + i) for i, k in enumerate(names)])
    for k in ("conv_final.weight", "conv_final.bias", "upconv0.weight", "upconv0.bias",
              "decoder1.4.weight", "decoder1.4.bias", "bn1.weight", "input_conv.weight",
              "enc4.2.bn2.weight", "upconv4.bias"):
        out["grad/" + k] = gr[k].grad.numpy().copy()
    bref = dict(ref.named_buffers()); borc = dict(orc.named_buffers())
    for k in bufnames:
        assert torch.equal(bref[k], borc[k]), k
    out["buf_proj_after_fwd"] = np.array([_proj(bref[k].float(), 9000 + i) for i, k in enumerate(bufnames)])
    out["running_mean/bn1"] = bref["bn1.running_mean"].numpy().copy()
    out["running_var/bn1"] = bref["bn1.running_var"].numpy().copy()
    opt_ref.step(); opt_orc.step()
    for k in names:
        assert torch.equal(gr[k], go[k]), k
    out["param_proj_after_step"] = np.array([_proj(gr[k].detach(), 8000 + i) for i, k in enumerate(names)])
    with torch.no_grad():
        mr = ref_utils.calculate_metrics(torch.sigmoid(lr_), m)
        mo = oracle.calculate_metrics(torch.sigmoid(lo_), m)
    assert mr == mo
    out["metrics_keys"] = np.array(sorted(mr))
    out["metrics_vals"] = np.array([mr[k] for k in sorted(mr)])

    # eval-mode logits from the closed-form running statistics
    ref.load_state_dict(sd); orc.load_state_dict(sd)
    ref.eval(); orc.eval()
    with torch.no_grad():
        le = ref(x); lo = orc(x)
    assert torch.equal(le, lo)
    out["logits_eval"] = le.numpy()

    # train_epoch / evaluate through the reference's own train.py on a 2-batch loader
    ref.load_state_dict(sd); orc.load_state_dict(sd)
    loader = [(x[:2], m[:2]), (x[2:], m[2:])]
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
    opt_orc = oracle.make_adam(orc)
    er = ref_train.train_epoch(ref, loader, opt_ref, crit_ref, torch.device("cpu"))
    eo = oracle.train_epoch(orc, loader, opt_orc, crit_orc, torch.device("cpu"))
    assert dict(er) == dict(eo), (er, eo)
    vr = ref_train.evaluate(ref, loader, torch.device("cpu"), crit_ref)
    vo = oracle.evaluate(orc, loader, torch.device("cpu"), crit_orc)
    assert dict(vr) == dict(vo)
    ek = sorted(er)
    out["epoch_keys"] = np.array(ek)
    out["train_epoch_vals"] = np.array([er[k] for k in ek])
    out["evaluate_vals"] = np.array([vr[k] for k in sorted(vr)])
    np.savez_compressed(os.path.join(HERE, "base64.npz"), **out)
    print("base64.npz: params", n_params, "bce", out["loss_bce"])

    # ---------------- mask threshold + metric edge cases ----------------
    thr = np.array([0x33C00001], np.uint32).view(np.float32)[0]
    bits = np.arange(0x33BFFFF0, 0x33C00010, dtype=np.uint32)
    vals = np.concatenate([bits.view(np.float32), -bits.view(np.float32),
                           np.array([0.0, -0.0, 1e-30, 1e-8, 8.9e-8, 9e-8, 1.0, -1.0, 30.0, -30.0,
                                     np.inf, -np.inf], np.float32)])
    t = torch.from_numpy(vals)
    mask_ref = (torch.sigmoid(t) > 0.5).numpy()
    assert np.array_equal(mask_ref, vals >= thr), "threshold rule changed in this torch build"
    edge = {}
    cases = {
        "empty_both": (np.zeros(64, np.float32), np.zeros(64, np.float32)),
        "all_fg": (np.ones(64, np.float32), np.ones(64, np.float32)),
        "pred_only": (np.ones(64, np.float32), np.zeros(64, np.float32)),
        "half": (np.r_[np.ones(32), np.zeros(32)].astype(np.float32), np.r_[np.ones(16), np.zeros(48)].astype(np.float32)),
    }
    for k, (p, g) in cases.items():
        r = ref_utils.calculate_metrics(torch.from_numpy(p), torch.from_numpy(g))
        edge[k] = np.array([r[kk] for kk in sorted(r)])
    np.savez_compressed(os.path.join(HERE, "mask_metrics.npz"), logits=vals, mask=mask_ref,
                        metric_keys=np.array(sorted(r)), **{"edge/" + k: v for k, v in edge.items()})

    # ---------------- losses on random logits ----------------
    g = torch.Generator().manual_seed(5)
    lg = torch.randn(3, 1, 32, 32, generator=g) * 3
    tg = (torch.rand(3, 1, 32, 32, generator=g) < 0.3).float()
    lo_out = {"logits": lg.numpy(), "target": tg.numpy()}
    for name in ("bce", "dice", "combo"):
        for alpha in ((0.5, 0.3) if name == "combo" else (None,)):
            cfg = {"loss_fn": name}
            if alpha is not None:
                cfg["loss_alpha"] = alpha
            z = lg.clone().requires_grad_(True)
            val = ref_losses.get_loss_function(cfg)(z, tg)
            val.backward()
            z2 = lg.clone().requires_grad_(True)
            v2 = oracle.get_loss_function(cfg)(z2, tg)
            v2.backward()
            assert torch.equal(val, v2) and torch.equal(z.grad, z2.grad)
            key = name if alpha is None else f"{name}_{alpha}"
            lo_out["val/" + key] = np.float32(val.item())
            lo_out["grad/" + key] = z.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "losses.npz"), **lo_out)

    # ---------------- tiny config from the reference's block vocabulary ----------------
    tiny = oracle.TinyUNet()
    ref_blocks = [am.UNetWithBackbone._decoder_block(None, ci, co) for ci, co in ((1, 8), (8, 16), (16, 8))]
    tsd = oracle.closed_form_state_dict(tiny, seed=3)
    tiny.load_state_dict(tsd)
    for blk, mine in zip(ref_blocks, (tiny.enc, tiny.mid, tiny.dec)):
        assert [tuple(p.shape) for p in blk.state_dict().values()] == \
            [tuple(p.shape) for p in mine.state_dict().values()]
        blk.load_state_dict(mine.state_dict())
    xt, mt = syn.synthetic_cells(4, 64, 64, seed=1234)
    xt = torch.from_numpy(xt)
    tiny.train()
    for blk in ref_blocks:
        blk.train()
    e_ref = ref_blocks[0](xt)
    assert torch.equal(e_ref, tiny.enc(xt))
    tiny.load_state_dict(tsd)
    lt = tiny(xt)
    lt_loss = oracle.bce_with_logits(lt, torch.from_numpy(mt))
    lt_loss.backward()
    tout = {"x": xt.numpy(), "masks": mt, "logits": lt.detach().numpy(), "loss_bce": np.float32(lt_loss.item())}
    for k, p in tiny.named_parameters():
        tout["grad/" + k] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "tiny64.npz"), **tout)

    # ---------------- attention decoder (use_attention=True, the reference default) ----------------
    torch.manual_seed(0)
    ref = am.UNetWithBackbone(n_classes=1, backbone="resnet34", pretrained=False, use_attention=True)
    orc = oracle.ReferenceUNet(use_attention=True)
    rk = [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
    ok = [(k, tuple(v.shape)) for k, v in orc.state_dict().items()]
    assert rk == ok, "attention state_dict layout differs from the reference"
    sd = oracle.closed_form_state_dict(orc, seed=0)
    ref.load_state_dict(sd); orc.load_state_dict(sd)
    ref.train(); orc.train()
    lr_ = ref(x); lo_ = orc(x)
    assert torch.equal(lr_, lo_), "attention: oracle logits != reference logits"
    loss_r = ref_losses.get_loss_function({"loss_fn": "bce"})(lr_, m)
    loss_o = oracle.get_loss_function({"loss_fn": "bce"})(lo_, m)
    assert torch.equal(loss_r, loss_o)
    loss_r.backward(); loss_o.backward()
    gr = dict(ref.named_parameters()); go = dict(orc.named_parameters())
    for k in gr:
        assert torch.equal(gr[k].grad, go[k].grad), k
    aout = {"x": x_np, "masks": m_np, "n_params": np.int64(sum(p.numel() for p in ref.parameters())),
            "logits_train": lr_.detach().numpy(), "loss_bce": np.float32(loss_r.item())}
    for k in gr:
        if k.startswith(("attention", "ch_attention", "conv_final", "upconv0")):
            aout["grad/" + k] = gr[k].grad.numpy().copy()
    bref = dict(ref.named_buffers())
    for k in bref:
        if k.startswith("attention") and not k.endswith("num_batches_tracked"):
            aout["buf/" + k] = bref[k].numpy().copy()
    ref.load_state_dict(sd); orc.load_state_dict(sd)
    ref.eval(); orc.eval()
    with torch.no_grad():
        le = ref(x); lo = orc(x)
    assert torch.equal(le, lo)
    aout["logits_eval"] = le.numpy()
    np.savez_compressed(os.path.join(HERE, "attn64.npz"), **aout)
    print("attn64.npz: params", int(aout["n_params"]), "bce", aout["loss_bce"])
    resnet50_fixture(am, ref_losses, oracle, syn)
    print("fixtures written; oracle == reference on every case")


if __name__ == "__main__":
    main()
