"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every
symbol include/unet_hip.h declares, the native plan reproduces the reference
parameter table, and the product path refuses to fall back to the CPU."""
import copy
import ctypes
import importlib
import os
import re

import numpy as np
import pytest
import torch

import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "unet_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(unet_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(pkg):
    lib_mod = importlib.import_module("image-segmentation-project_amd._lib")
    lib = lib_mod.load()
    syms = _declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in lib_mod.SIGNATURES, f"{s} has no ctypes signature"
    assert b"gfx950" in lib.unet_version()


def test_plan_matches_reference_parameter_table(pkg):
    am = importlib.import_module("image-segmentation-project_amd.advanced_models")
    plan = am._Plan(4, 64, 64, 1, 1, torch.device("cpu"))
    ref = oracle.ReferenceUNet()
    names = [k for k, _ in ref.named_parameters()]
    assert plan.param_names == names
    assert plan.param_shapes == [tuple(p.shape) for _, p in ref.named_parameters()]
    offs = np.cumsum([0] + [p.numel() for p in ref.parameters()])[:-1]
    assert plan.param_offsets == list(offs)
    assert plan.grad_numel == 24339457
    # buckets tile the flat gradient buffer exactly, in backward order
    b = plan.buckets
    assert b[0][1] == plan.grad_numel and b[-1][0] == 0
    assert all(b[i][0] == b[i + 1][1] for i in range(len(b) - 1))


def test_attention_plan_and_module_match_reference_layout(pkg):
    """use_attention=True: native parameter table, BN/buffer order and the
    module's state_dict equal the reference layout (24,441,229 params)."""
    am = importlib.import_module("image-segmentation-project_amd.advanced_models")
    plan = am._Plan(4, 64, 64, 1, 1, torch.device("cpu"), attention=True)
    ref = oracle.ReferenceUNet(use_attention=True)
    assert plan.param_names == [k for k, _ in ref.named_parameters()]
    assert plan.param_shapes == [tuple(p.shape) for _, p in ref.named_parameters()]
    assert plan.grad_numel == 24441229
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=True)
    assert [(k, tuple(v.shape)) for k, v in m.state_dict().items()] == \
        [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
    b = plan.buckets
    assert b[0][1] == plan.grad_numel and b[-1][0] == 0


def test_algorithmic_flops_match_survey(pkg):
    am = importlib.import_module("image-segmentation-project_amd.advanced_models")
    plan = am._Plan(16, 512, 512, 1, 1, torch.device("cpu"))
    assert abs(plan.flops_fwd / 16 / 1e9 - 54.509) < 1e-3
    assert abs(plan.flops_train / 16 / 1e9 - 163.1165) < 1e-3  # 3 x fwd - stem dgrad
    hi = am._Plan(4, 1024, 1024, 1, 1, torch.device("cpu"))
    assert abs(hi.flops_train / 4 / 1e9 - 652.5) < 0.1


def test_plan_rejects_bad_shapes(pkg):
    am = importlib.import_module("image-segmentation-project_amd.advanced_models")
    with pytest.raises(RuntimeError, match="multiples of 32"):
        am._Plan(2, 100, 100, 1, 1, torch.device("cpu"))


def test_module_state_dict_equals_reference_layout(pkg):
    m = pkg.UNetWithBackbone(n_classes=1, backbone="resnet34", pretrained=False, use_attention=False)
    ref = oracle.ReferenceUNet()
    assert [(k, tuple(v.shape)) for k, v in m.state_dict().items()] == \
        [(k, tuple(v.shape)) for k, v in ref.state_dict().items()]
    sd = oracle.closed_form_state_dict(ref)
    m.load_state_dict(sd)
    m2 = copy.deepcopy(m)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    assert len(opt.param_groups[0]["params"]) == 152


def test_unsupported_configs_raise(pkg):
    with pytest.raises(NotImplementedError):
        pkg.UNetWithBackbone(backbone="densenet121", pretrained=False, use_attention=False)
    with pytest.raises(NotImplementedError):
        pkg.UNetWithBackbone(backbone="resnet50", pretrained=False, use_attention=False, width=2)
    with pytest.warns(RuntimeWarning):
        pkg.UNetWithBackbone(pretrained=True, use_attention=False)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_no_cpu_fallback(pkg):
    m = pkg.UNetWithBackbone(pretrained=False, use_attention=False)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 1, 64, 64))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pkg.BCELoss()(torch.zeros(4), torch.zeros(4))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pkg.calculate_metrics(torch.zeros(4), torch.zeros(4))


def test_loss_registry(pkg, capsys):
    assert isinstance(pkg.get_loss_function({}), pkg.ComboLoss)
    assert isinstance(pkg.get_loss_function({"loss_fn": "bce"}), pkg.BCELoss)
    d = pkg.get_loss_function({"loss_fn": "dice", "smooth": 2.0})
    assert isinstance(d, pkg.DiceLoss) and d.smooth == 2.0
    c = pkg.get_loss_function({"loss_fn": "nope", "loss_alpha": 0.3})
    assert isinstance(c, pkg.ComboLoss) and c.alpha == 0.3
    assert "Unknown loss function 'nope'" in capsys.readouterr().out
    with pytest.raises(NotImplementedError):
        pkg.get_loss_function({"loss_fn": "focal"})


def test_early_stopping_matches_reference_semantics(pkg):
    es = pkg.EarlyStopping(patience=2, min_delta=0.01)
    seq = [0.5, 0.505, 0.509, 0.6, 0.6]
    out = [es.step(v) for v in seq]
    assert out == [False, False, True, True, True]  # early_stop latches (utils.py:182-190)


def test_metrics_formula_matches_reference(pkg, golden):
    utils = importlib.import_module("image-segmentation-project_amd.utils")
    g = golden("mask_metrics.npz")
    keys = list(g["metric_keys"])
    cases = {"empty_both": (0, 0, 0, 64), "all_fg": (64, 0, 0, 0), "pred_only": (0, 64, 0, 0),
             "half": (16, 16, 0, 32)}
    for name, c in cases.items():
        m = utils.metrics_from_counts(*map(float, c))
        assert [m[k] for k in keys] == list(g["edge/" + name]), name


def test_synthetic_cells(pkg):
    x, m = pkg.synthetic_cells(2, 128, 128, seed=1234)
    assert x.shape == (2, 1, 128, 128) and x.dtype == np.float32
    assert x.min() >= 0 and x.max() <= 1
    assert set(np.unique(m)) <= {0.0, 1.0}
    x2, _ = pkg.synthetic_cells(2, 128, 128, seed=1234)
    assert np.array_equal(x, x2)


def test_importable_alias_and_reference_layout_modules(pkg):
    """`import image_segmentation_project_amd` and the reference's own flat module
    names (dropin/advanced_models.py, losses.py, train.py, utils.py) resolve to
    the same module objects as the hyphenated package."""
    import sys
    import image_segmentation_project_amd as amd
    assert amd is pkg
    from image_segmentation_project_amd.ddp import enable_data_parallel
    assert enable_data_parallel is pkg.ddp.enable_data_parallel
    sys.path.insert(0, os.path.join(REPO, "dropin"))
    try:
        for name, attrs in (("advanced_models", ["UNetWithBackbone"]),
                            ("losses", ["get_loss_function", "BCELoss", "DiceLoss", "ComboLoss"]),
                            ("train", ["train_epoch", "evaluate", "train_model", "quick_train"]),
                            ("utils", ["calculate_metrics", "get_device", "EarlyStopping"])):
            mod = importlib.import_module(name)
            for a in attrs:
                assert getattr(mod, a) is getattr(pkg, a), (name, a)
    finally:
        sys.path.remove(os.path.join(REPO, "dropin"))
        for name in ("advanced_models", "losses", "train", "utils"):
            sys.modules.pop(name, None)


def test_loss_scratch_length_matches_header(pkg):
    """losses.py / utils.py size the loss partial scratch from _lib.LOSS_SCRATCH_LEN
    and pass its length; the library checks it against UNET_LOSS_SCRATCH_LEN and
    writes exactly 8 doubles to sums8 (an 8-double sums8 buffer is
    safe, a short scratch fails loudly)."""
    lib_mod = importlib.import_module("image-segmentation-project_amd._lib")
    src = open(os.path.join(REPO, "include", "unet_hip.h")).read()
    m = re.search(r"#define\s+UNET_LOSS_SCRATCH_LEN\s+\(8 \* (\d+)\)", src)
    assert m, "UNET_LOSS_SCRATCH_LEN not found in include/unet_hip.h"
    assert lib_mod.LOSS_SCRATCH_LEN == 8 * int(m.group(1))
    sums, scratch = lib_mod.loss_buffers("cpu")
    assert sums.numel() == 8 and scratch.numel() == lib_mod.LOSS_SCRATCH_LEN


def test_loss_short_scratch_is_rejected(pkg):
    """A scratch shorter than UNET_LOSS_SCRATCH_LEN is refused before any launch
    (no device memory is touched, so this runs without a GPU)."""
    lib_mod = importlib.import_module("image-segmentation-project_amd._lib")
    lib = lib_mod.load()
    rc = lib.unet_loss_forward(None, None, 16, 0, 0.5, 1.0, 8, 16, 8 * 255, None, None)
    assert rc != 0 and b"UNET_LOSS_SCRATCH_LEN" in lib.unet_last_error()
    rc = lib.unet_mask_metrics(None, None, 16, 0, 8, None, lib_mod.LOSS_SCRATCH_LEN, None)
    assert rc != 0
