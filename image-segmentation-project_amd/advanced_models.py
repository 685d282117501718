"""``UNetWithBackbone`` for MI355X — same constructor, forward and state_dict as
/root/reference/advanced_models.py:64-357 (resnet34 encoder, no attention).

The module tree below exists only to own parameters and buffers under the
reference's names (``input_conv``, ``bn1``, ``enc1..4`` = torchvision ResNet34
``layer1..4``, ``upconv4..0``, ``decoder4..1`` = ``_decoder_block`` Sequentials,
``conv_final``), so ``state_dict()``/``load_state_dict()``/``copy.deepcopy`` and a
caller-built ``torch.optim.Adam(model.parameters())`` behave exactly as with the
reference (``train.py:207-226``, ``cross_validation.py:84-100``).  ``forward``
never runs these submodules: it hands raw device pointers to the native
executor in ``libunet_hip.so`` (bf16 NHWC activations, MFMA implicit-GEMM
convolutions, fused BN/ReLU/residual kernels) through one autograd Function.
"""
from __future__ import annotations

import ctypes
import warnings

import torch
import torch.nn as nn

from . import _lib


class _BasicBlock(nn.Module):
    """Parameter container with torchvision BasicBlock names (conv1/bn1/conv2/bn2/downsample)."""

    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        self.stride = stride


class _Bottleneck(nn.Module):
    """Parameter container with torchvision Bottleneck names (resnet50 encoder,
    advanced_models.py:102-117): conv1 1x1 / bn1 / conv2 3x3 (stride) / bn2 /
    conv3 1x1 (x4) / bn3 / downsample."""

    def __init__(self, cin: int, planes: int, stride: int):
        super().__init__()
        cout = planes * 4
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        self.stride = stride


def _layer(cin, cout, n, stride):
    return nn.Sequential(_BasicBlock(cin, cout, stride), *[_BasicBlock(cout, cout, 1) for _ in range(n - 1)])


def _layer50(cin, planes, n, stride):
    return nn.Sequential(_Bottleneck(cin, planes, stride), *[_Bottleneck(planes * 4, planes, 1) for _ in range(n - 1)])


def _decoder_block(cin, cout):
    # advanced_models.py:197-205 layout: indices 0,1,3,4 carry state
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                         nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class _AttentionGate(nn.Module):
    """Parameter container of ``AttentionGate`` (advanced_models.py:7-40); computed natively."""

    def __init__(self, f_g, f_l, f_int):
        super().__init__()
        self.W_g = nn.Sequential(nn.Conv2d(f_g, f_int, 1, bias=True), nn.BatchNorm2d(f_int))
        self.W_x = nn.Sequential(nn.Conv2d(f_l, f_int, 1, bias=True), nn.BatchNorm2d(f_int))
        self.psi = nn.Sequential(nn.Conv2d(f_int, 1, 1, bias=True), nn.BatchNorm2d(1), nn.Sigmoid())
        self.relu = nn.ReLU(inplace=True)


class _ChannelAttention(nn.Module):
    """Parameter container of ``ChannelAttention`` (advanced_models.py:43-61); computed natively."""

    def __init__(self, c, reduction_ratio=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.fc = nn.Sequential(nn.Conv2d(c, c // reduction_ratio, 1, bias=False), nn.ReLU(inplace=True),
                                nn.Conv2d(c // reduction_ratio, c, 1, bias=False))
        self.sigmoid = nn.Sigmoid()


class _Plan:
    """Owns one native plan (per input shape) and its persistent workspace."""

    def __init__(self, n, h, w, width, n_classes, device, attention=False, backbone=34, fp8=False):
        lib = _lib.load()
        cfg = _lib.UnetConfig(n, h, w, width, n_classes, 1e-5, 0.1, 1 if attention else 0, backbone,
                              1 if fp8 else 0)
        handle = ctypes.c_void_p()
        _lib.check(lib.unet_plan_create(ctypes.byref(cfg), ctypes.byref(handle)), "unet_plan_create")
        self.lib, self.handle = lib, handle
        self.shape = (n, h, w)
        ws_bytes = lib.unet_plan_workspace_bytes(handle)
        self.workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
        self.grad_numel = lib.unet_plan_grad_numel(handle)
        nparam = lib.unet_plan_num_params(handle)
        buf = ctypes.create_string_buffer(256)
        self.param_names, self.param_offsets, self.param_shapes = [], [], []
        shape = (ctypes.c_int64 * 4)()
        for i in range(nparam):
            _lib.check(lib.unet_plan_param_name(handle, i, buf, 256), "param_name")
            self.param_names.append(buf.value.decode())
            nd = lib.unet_plan_param_shape(handle, i, shape)
            self.param_shapes.append(tuple(shape[k] for k in range(nd)))
            self.param_offsets.append(lib.unet_plan_param_offset(handle, i))
        self.buckets = []
        b0, b1 = ctypes.c_int64(), ctypes.c_int64()
        for b in range(lib.unet_plan_num_buckets(handle)):
            _lib.check(lib.unet_plan_bucket_range(handle, b, ctypes.byref(b0), ctypes.byref(b1)), "bucket_range")
            self.buckets.append((b0.value, b1.value))
        self.flops_train = lib.unet_plan_flops(handle, 1)
        self.flops_fwd = lib.unet_plan_flops(handle, 0)
        self.generation = 0
        self.pins = 0  # GraphedTrainStep captures holding this plan's workspace
        self.last_used = 0

    def profile(self, on: bool):
        _lib.check(self.lib.unet_profile_enable(self.handle, 1 if on else 0), "unet_profile_enable")

    def profile_report(self):
        """[(name, ms, flops, kernel)] for every launch recorded since profile(True);
        kernel = the conv kernel's template instance (as rocprofv3 names it) for
        conv launches, "" otherwise."""
        n = self.lib.unet_profile_report(self.handle, None, 0)
        if n < 0:
            _lib.check(1, "unet_profile_report")
        buf = ctypes.create_string_buffer(n + 16)
        self.lib.unet_profile_report(self.handle, buf, n + 16)
        out = []
        for line in buf.value.decode().splitlines():
            name, ms, fl, kern = (line.split("\t") + [""])[:4]
            out.append((name, float(ms), float(fl), kern))
        return out

    def tensor_views(self):
        """name -> NCHW float32 copy of a bf16 NHWC workspace tensor (tests / debugging)."""
        lib, h = self.lib, self.handle
        info = (ctypes.c_int64 * 5)()
        buf = ctypes.create_string_buffer(128)
        out = {}
        n = self.shape[0]
        ws = self.workspace.view(torch.bfloat16)
        for i in range(lib.unet_plan_num_tensors(h)):
            _lib.check(lib.unet_plan_tensor_info(h, i, buf, 128, info), "tensor_info")
            off, ld, c, hh, ww = (int(v) for v in info)
            t = ws.as_strided((n, hh, ww, c), (hh * ww * ld, ww * ld, ld, 1), off // 2)
            out[buf.value.decode()] = t.permute(0, 3, 1, 2).float()
        return out

    def __del__(self):
        try:
            if self.handle:
                self.lib.unet_plan_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class _UNetFunction(torch.autograd.Function):
    """logits = UNet(x; params).  Backward runs the whole native backward pass and
    returns every parameter gradient as a view of one flat fp32 buffer."""

    @staticmethod
    def forward(ctx, model, x, *params):
        plan = model._plan_for(x)
        logits = model._run_forward(plan, x, training=True)
        ctx.model = model
        ctx.plan = plan
        ctx.generation = plan.generation
        ctx.save_for_backward(x)
        return logits

    @staticmethod
    def backward(ctx, grad_logits):
        (x,) = ctx.saved_tensors
        model, plan = ctx.model, ctx.plan
        if plan.generation != ctx.generation:
            raise RuntimeError("UNetWithBackbone: another forward overwrote the saved activations "
                               "before backward (one forward per backward on the same input shape)")
        grads = model._run_backward(plan, x, grad_logits.contiguous())
        views = [grads[o:o + p.numel()].view_as(p) for o, p in zip(plan.param_offsets, model._param_list)]
        return (None, None, *views)


class UNetWithBackbone(nn.Module):
    """Drop-in for ``advanced_models.UNetWithBackbone`` (resnet34 or resnet50,
    with or without attention).

    ``width`` is a build extension (1 = reference channels; resnet34 only).
    ``backbone='resnet50'`` builds the Bottleneck encoder (256..2048 channels)
    and its decoder (advanced_models.py:102-130,158-159); 'densenet121' is not
    runnable in the reference and raises
    ``NotImplementedError``.  ``use_attention=True`` (the reference default)
    adds the AttentionGate / ChannelAttention decoder (advanced_models.py:7-61).
    ``fp8=True`` (build extension, BASELINE configs[4] "Wide fp8"; resnet34
    without attention): forward convs with >= 128 input channels run on the
    fp8 e4m3 block-scaled MFMA with per-tensor delayed scaling; BN, the loss
    and the whole backward stay bf16/fp32.
    """

    def __init__(self, n_classes=1, backbone="resnet34", pretrained=True, use_attention=True, width=1, fp8=False):
        super().__init__()
        if fp8 and (backbone != "resnet34" or use_attention):
            raise NotImplementedError("fp8=True is built for the resnet34 U-Net without attention")
        self.fp8 = bool(fp8)
        if backbone not in ("resnet34", "resnet50"):
            raise NotImplementedError(f"backbone={backbone!r}: 'resnet34' and 'resnet50' are built for MI355X "
                                      "(densenet121 is broken in the reference, SURVEY.md §2 row 1)")
        if backbone == "resnet50" and width != 1:
            raise NotImplementedError("width != 1 is a resnet34 build extension")
        if n_classes != 1:
            raise NotImplementedError("n_classes must be 1 (binary segmentation, advanced_models.py:160)")
        if pretrained:
            warnings.warn("pretrained=True needs ImageNet weights from the network (unavailable offline); "
                          "the encoder keeps its random init — load a state_dict instead", RuntimeWarning)
        self.use_attention = use_attention
        self.backbone_name = backbone
        self._backbone_id = 50 if backbone == "resnet50" else 34
        self.width = width
        c0 = 64 * width
        self.input_conv = nn.Conv2d(1, c0, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(c0)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        if backbone == "resnet50":  # advanced_models.py:102-130
            ch = [256, 512, 1024, 2048]
            self.enc1 = _layer50(64, 64, 3, 1)
            self.enc2 = _layer50(256, 128, 4, 2)
            self.enc3 = _layer50(512, 256, 6, 2)
            self.enc4 = _layer50(1024, 512, 3, 2)
            up1, d1 = 64, 64
            att = [(1024, 1024, 512), (512, 512, 256), (256, 256, 128), (64, 64, 32)]
        else:  # advanced_models.py:72-100
            ch = [c0, 2 * c0, 4 * c0, 8 * c0]
            self.enc1 = _layer(ch[0], ch[0], 3, 1)
            self.enc2 = _layer(ch[0], ch[1], 4, 2)
            self.enc3 = _layer(ch[1], ch[2], 6, 2)
            self.enc4 = _layer(ch[2], ch[3], 3, 2)
            up1, d1 = c0 // 2, c0 // 2
            att = [(ch[2], ch[2], ch[1]), (ch[1], ch[1], ch[0]), (ch[0], ch[0], c0 // 2), (c0 // 2, c0, c0 // 2)]
        self.upconv4 = nn.ConvTranspose2d(ch[3], ch[2], kernel_size=2, stride=2)
        self.decoder4 = _decoder_block(2 * ch[2], ch[2])
        self.upconv3 = nn.ConvTranspose2d(ch[2], ch[1], kernel_size=2, stride=2)
        self.decoder3 = _decoder_block(2 * ch[1], ch[1])
        self.upconv2 = nn.ConvTranspose2d(ch[1], ch[0], kernel_size=2, stride=2)
        self.decoder2 = _decoder_block(2 * ch[0], ch[0])
        self.upconv1 = nn.ConvTranspose2d(ch[0], up1, kernel_size=2, stride=2)
        self.decoder1 = _decoder_block(c0 + up1, d1)
        self.upconv0 = nn.ConvTranspose2d(d1, c0 // 4, kernel_size=2, stride=2)
        self.conv_final = nn.Conv2d(c0 // 4, n_classes, kernel_size=1)
        if use_attention:  # advanced_models.py:163-183, registered after conv_final
            for lvl, (fg, fl, fi) in zip((4, 3, 2, 1), att):
                setattr(self, f"attention{lvl}", _AttentionGate(fg, fl, fi))
            for lvl, c in zip((4, 3, 2, 1), (ch[2], ch[1], ch[0], d1)):
                setattr(self, f"ch_attention{lvl}", _ChannelAttention(c))
        self._plans = {}
        self.max_plans = 3  # unpinned native plans (input shapes) kept alive
        self._use_clock = 0
        self._ddp = None  # set by ddp.enable_data_parallel

    # ------------------------------------------------------------------ plumbing
    def __getstate__(self):  # deepcopy / pickle: native plans are rebuilt lazily
        state = self.__dict__.copy()
        state["_plans"] = {}
        return state

    @property
    def _last_plan(self):
        """The most recently used native plan (tests / profiling)."""
        return max(self._plans.values(), key=lambda pl: pl.last_used)

    @property
    def _param_list(self):
        return [p for _, p in self.named_parameters()]

    def _plan_for(self, x) -> _Plan:
        if x.dim() != 4 or x.shape[1] != 1:
            raise ValueError(f"expected input [N,1,H,W], got {tuple(x.shape)}")
        n, _, h, w = x.shape
        key = (n, h, w, x.device)
        plan = self._plans.get(key)
        if plan is None:
            plan = _Plan(n, h, w, self.width, 1, x.device, self.use_attention, self._backbone_id, self.fp8)
            names = [k for k, _ in self.named_parameters()]
            if names != plan.param_names:
                raise RuntimeError("native parameter table does not match the module's named_parameters()")
            for p, s in zip(self._param_list, plan.param_shapes):
                if tuple(p.shape) != s:
                    raise RuntimeError(f"parameter shape mismatch {tuple(p.shape)} vs {s}")
            # a small LRU of shapes (a ragged last batch or another val batch size
            # must not rebuild the big plan every epoch); pinned plans (captured
            # by a GraphedTrainStep) are never evicted
            live = sorted((k for k, v in self._plans.items() if v.pins == 0),
                          key=lambda k: self._plans[k].last_used)
            while len(live) >= self.max_plans:
                self._plans.pop(live.pop(0))
            self._plans[key] = plan
        self._use_clock += 1
        plan.last_used = self._use_clock
        return plan

    def _pointer_arrays(self):
        params = self._param_list
        for p in params:
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                raise RuntimeError("UNetWithBackbone parameters must be contiguous fp32 on the GPU")
        pa = (ctypes.c_void_p * len(params))(*[p.data_ptr() for p in params])
        bufs = [b for _, b in self.named_buffers()]
        ba = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
        return pa, ba

    def _run_forward(self, plan, x, training: bool):
        _lib.require_gpu(x)
        x = x.contiguous().float()
        n, _, h, w = x.shape
        logits = torch.empty((n, 1, h, w), dtype=torch.float32, device=x.device)
        pa, ba = self._pointer_arrays()
        plan.generation += 1
        rc = plan.lib.unet_forward(plan.handle, x.data_ptr(), pa, ba, plan.workspace.data_ptr(), logits.data_ptr(),
                                   1 if training else 0, _lib.stream_handle(x.device))
        _lib.check(rc, "unet_forward")  # training: it also adds 1 to every num_batches_tracked
        return logits

    def _run_backward(self, plan, x, grad_logits):
        grads = torch.empty(plan.grad_numel, dtype=torch.float32, device=x.device)
        pa, _ = self._pointer_arrays()
        rc = plan.lib.unet_backward(plan.handle, x.contiguous().data_ptr(), grad_logits.data_ptr(), pa,
                                    plan.workspace.data_ptr(), grads.data_ptr(), _lib.stream_handle(x.device))
        _lib.check(rc, "unet_backward")
        if self._ddp is not None:
            self._ddp.reduce(plan, grads)
        return grads

    # ------------------------------------------------------------------ API
    def forward(self, x, return_features=False):
        if return_features:
            raise NotImplementedError("return_features (advanced_models.py:352-356) is not on the hot path")
        _lib.require_gpu(x)
        x = x.contiguous().float()
        if self.training:
            if torch.is_grad_enabled():
                return _UNetFunction.apply(self, x, *self._param_list)
            return self._run_forward(self._plan_for(x), x, training=True)
        with torch.no_grad():
            return self._run_forward(self._plan_for(x), x, training=False)

    def step_flops(self, x_shape, training=True) -> float:
        """Algorithmic FLOPs of one step at input shape [N,1,H,W]."""
        n, _, h, w = x_shape
        lib = _lib.load()
        cfg = _lib.UnetConfig(n, h, w, self.width, 1, 1e-5, 0.1, 1 if self.use_attention else 0, self._backbone_id,
                              1 if self.fp8 else 0)
        handle = ctypes.c_void_p()
        _lib.check(lib.unet_plan_create(ctypes.byref(cfg), ctypes.byref(handle)), "unet_plan_create")
        try:
            return lib.unet_plan_flops(handle, 1 if training else 0)
        finally:
            lib.unet_plan_destroy(handle)
