"""Fused Adam for MI355X — a drop-in for the ``torch.optim.Adam`` the reference
builds (/root/reference/train.py:331-335: ``torch.optim.Adam(model.parameters(),
lr=config['learning_rate'], weight_decay=config['weight_decay'])``; called once
per batch at train.py:49).

Same constructor, ``param_groups``, ``state`` keys (``step``, ``exp_avg``,
``exp_avg_sq``), ``state_dict``/``load_state_dict`` and per-element math as
torch's Adam with coupled L2 weight decay (torch/optim/adam.py
``_single_tensor_adam``).  What differs is where it runs: each parameter group
lives in four flat fp32 buffers (parameters, gradients, first and second
moments) and one step is two launches of ``unet_adam_step``
(``csrc/optim.hip``) instead of ~300 small foreach launches.

* Parameters are re-homed once into one flat buffer per group (``p.data``
  becomes a view; the ``nn.Parameter`` objects, and so the module, are
  unchanged).  The U-Net's backward already returns every gradient as a view of
  one flat buffer in parameter order, so the step reads gradients in place;
  gradients laid out any other way are first gathered with ``torch.cat``.
* Step counters live on the device (graph-capturable; ``capturable`` is
  always True).  While every parameter of a group has taken the same number of
  steps they share one counter (``state[p]['step']`` is that tensor) and a step
  is one launch over the group.  Parameters whose ``.grad`` is None are skipped
  as torch skips them; from then on each parameter keeps its own counter (and
  bias correction, exactly as torch's per-parameter ``state['step']``) and is
  stepped by its own launch, until the counts agree again.
* ``lr`` / ``weight_decay`` are read from ``param_groups`` at every call; under
  HIP-graph capture they are fixed at capture time.
* ``amsgrad``, ``maximize`` and ``differentiable`` are not on the reference path
  and raise ``NotImplementedError``.
"""
from __future__ import annotations

import torch

from . import _lib


def _chain_ok(tensors, base) -> bool:
    """True when `tensors` lie back to back, in order, from base.data_ptr()."""
    ptr = base.data_ptr()
    for t in tensors:
        if t.data_ptr() != ptr or not t.is_contiguous():
            return False
        ptr += t.numel() * 4
    return True


class _FlatGroup:
    def __init__(self, params, state):
        dev = params[0].device
        for p in params:
            if p.device != dev or p.dtype != torch.float32:
                raise RuntimeError("fused Adam: every parameter of a group must be fp32 on one GPU")
        self.params = list(params)
        self.numels = [p.numel() for p in params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.total = off
        # parameters: re-home into one flat buffer unless they already are one
        base = params[0].data
        flat = None
        if base.storage_offset() == 0 and base.untyped_storage().nbytes() >= self.total * 4 and \
                _chain_ok([p.data for p in params], base):
            flat = torch.as_strided(base, (self.total,), (1,), 0)
        if flat is None:
            flat = torch.empty(self.total, dtype=torch.float32, device=dev)
            for p, o, n in zip(params, self.offsets, self.numels):
                flat[o:o + n].copy_(p.data.reshape(-1))
                p.data = flat[o:o + n].view_as(p)
        self.pflat = flat
        self.m = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.coef = torch.zeros(3, dtype=torch.float32, device=dev)  # step, step_size, sqrt(bc2)
        # per-parameter counters (used once the parameters' step counts differ)
        self.pcoef = torch.zeros(len(params), 3, dtype=torch.float32, device=dev)
        self.counts = []
        for p, o, n in zip(params, self.offsets, self.numels):  # carry over existing / loaded state
            st = state.get(p)
            if st and "exp_avg" in st:
                self.m[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self.v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                self.counts.append(int(float(st["step"])))
            else:
                self.counts.append(0)
        for i, (p, o, n) in enumerate(zip(params, self.offsets, self.numels)):
            state[p] = {"exp_avg": self.m[o:o + n].view_as(p), "exp_avg_sq": self.v[o:o + n].view_as(p)}
        self.state = state
        self.uniform = None
        self._set_mode(len(set(self.counts)) <= 1)
        self.gstage = None

    def _set_mode(self, uniform: bool):
        """uniform: one shared device counter; else one counter row per parameter."""
        if uniform == self.uniform:
            return
        if uniform:
            self.coef[0] = float(self.counts[0] if self.counts else 0)
            for p in self.params:
                self.state[p]["step"] = self.coef[0]
        else:
            if self.uniform:
                # leaving the shared counter: it is the truth (HIP-graph replays
                # of the step advance it on the device without touching counts)
                self.counts = [int(self.coef[0].item())] * len(self.params)
            self.pcoef[:, 0] = torch.tensor(self.counts, dtype=torch.float32)
            for i, p in enumerate(self.params):
                self.state[p]["step"] = self.pcoef[i, 0]
        self.uniform = uniform

    def valid(self, params, state) -> bool:
        if len(params) != len(self.params) or any(a is not b for a, b in zip(params, self.params)):
            return False
        if not _chain_ok([p.data for p in params], self.pflat):
            return False
        st = state.get(params[0])
        return bool(st) and st.get("exp_avg") is not None and \
            st["exp_avg"].data_ptr() == self.m.data_ptr()


class Adam(torch.optim.Optimizer):
    """``torch.optim.Adam`` signature; see the module docstring."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=True, differentiable=False, fused=None):
        if isinstance(lr, torch.Tensor):
            lr = float(lr)
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad or maximize or differentiable:
            raise NotImplementedError("fused Adam: amsgrad / maximize / differentiable are not on the reference "
                                      "path (train.py:331-335); use torch.optim.Adam for them")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=True, differentiable=False, fused=None)
        super().__init__(params, defaults)
        self._flat = {}

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat = {}  # rebuilt from the loaded per-parameter state at the next step

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for gi, group in enumerate(self.param_groups):
            params = group["params"]
            if not params:
                continue
            with_grad = [p for p in params if p.grad is not None]
            if not with_grad:
                continue
            _lib.require_gpu(params[0])
            fg = self._flat.get(gi)
            if fg is None or not fg.valid(params, self.state):
                fg = self._flat[gi] = _FlatGroup(params, self.state)
            beta1, beta2 = group["betas"]
            lr, eps, wd = float(group["lr"]), float(group["eps"]), float(group["weight_decay"])
            stream = _lib.stream_handle(params[0].device)
            full = len(with_grad) == len(params)
            if full and fg.uniform:
                grads = [p.grad for p in params]
                if grads[0].storage_offset() >= 0 and _chain_ok(grads, grads[0]):
                    gptr = grads[0].data_ptr()
                else:
                    fg.gstage = torch.cat([g.reshape(-1) for g in grads])
                    gptr = fg.gstage.data_ptr()
                _lib.check(lib.unet_adam_step(fg.pflat.data_ptr(), gptr, fg.m.data_ptr(), fg.v.data_ptr(),
                                              fg.coef.data_ptr(), fg.total, lr, beta1, beta2, eps, wd, 1, stream),
                           "unet_adam_step")
                fg.counts = [c + 1 for c in fg.counts]
            else:  # torch skips parameters without gradients; each keeps its own step count
                fg._set_mode(False)
                for i, (p, o, n) in enumerate(zip(params, fg.offsets, fg.numels)):
                    if p.grad is None:
                        continue
                    g = p.grad.contiguous()
                    _lib.check(lib.unet_adam_step(fg.pflat[o:].data_ptr(), g.data_ptr(), fg.m[o:].data_ptr(),
                                                  fg.v[o:].data_ptr(), fg.pcoef[i].data_ptr(), n, lr, beta1,
                                                  beta2, eps, wd, 1, stream), "unet_adam_step")
                    fg.counts[i] += 1
                if len(set(fg.counts)) == 1:
                    fg._set_mode(True)
        return loss
