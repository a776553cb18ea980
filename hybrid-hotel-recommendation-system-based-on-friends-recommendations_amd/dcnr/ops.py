"""Loss and optimizer on libdcnr: drop-ins for ``nn.BCEWithLogitsLoss``
(train.py:206, 224) and ``torch.optim.AdamW`` / ``Adam`` (train.py:201-204,
226)."""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from . import _lib


def bce_with_logits(logits: torch.Tensor, target: torch.Tensor, want_grad: bool = True,
                    grad_scale: float = 1.0):
    """Mean BCE-with-logits on the device.  Returns (loss 0-d tensor, dlogits or None)
    with dlogits = grad_scale * (sigmoid(z) - y) / B."""
    lib = _lib.load()
    z = logits.reshape(-1).to(torch.float32).contiguous()
    y = target.reshape(-1).to(torch.float32).contiguous()
    if z.device.type != 'cuda':
        raise RuntimeError("dcnr.bce_with_logits runs on the HIP device only")
    B = z.shape[0]
    ws = torch.empty(int(lib.dcnr_bce_workspace_size()), dtype=torch.uint8, device=z.device)
    loss = torch.empty((), dtype=torch.float32, device=z.device)
    dz = torch.empty_like(z) if want_grad else None
    _lib.check(lib.dcnr_bce_with_logits(z.data_ptr(), y.data_ptr(), B, loss.data_ptr(),
                                        dz.data_ptr() if dz is not None else None,
                                        float(grad_scale), ws.data_ptr(), ws.numel(),
                                        _lib.stream_ptr(z.device)), "dcnr_bce_with_logits")
    return loss, dz


class _BCEFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        loss, dz = bce_with_logits(logits, target, want_grad=logits.requires_grad)
        ctx.shape = logits.shape
        ctx.save_for_backward(dz if dz is not None else torch.empty(0))
        return loss

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return (dz * g).reshape(ctx.shape), None


class BCEWithLogitsLoss(nn.Module):
    """nn.BCEWithLogitsLoss() (reduction='mean', no weights) on libdcnr."""

    def forward(self, input, target):
        if input.shape != target.shape:
            raise ValueError(f"Target size ({target.shape}) must be the same as input size "
                             f"({input.shape})")
        return _BCEFunction.apply(input, target)


class _FusedAdamBase(torch.optim.Optimizer):
    """Multi-tensor Adam/AdamW in ONE launch per group (dcnr_adam_step); same
    hyper-parameters, update rule and state keys (step, exp_avg, exp_avg_sq)
    as torch.optim, so optimizer state_dicts interchange."""

    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=None):
        if weight_decay is None:
            weight_decay = 1e-2 if self.decoupled else 0.0
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for group in self.param_groups:
            ps, gs, ms, vs, ns = [], [], [], [], []
            step_val = None
            for p in group['params']:
                if p.grad is None:
                    continue
                if p.device.type != 'cuda' or p.dtype != torch.float32 or not p.is_contiguous() \
                        or not p.grad.is_contiguous():
                    raise RuntimeError("dcnr fused Adam needs fp32 contiguous HIP tensors")
                if p.grad.is_sparse:
                    raise RuntimeError("dcnr fused Adam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st['step'] = torch.tensor(0.0)
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['step'] += 1
                s = int(st['step'].item())
                if step_val is not None and s != step_val:
                    # groups with mixed step counts: launch per distinct step
                    self._launch(lib, group, ps, gs, ms, vs, ns, step_val)
                    ps, gs, ms, vs, ns = [], [], [], [], []
                step_val = s
                ps.append(p); gs.append(p.grad); ms.append(st['exp_avg'])
                vs.append(st['exp_avg_sq']); ns.append(p.numel())
            if ps:
                self._launch(lib, group, ps, gs, ms, vs, ns, step_val)
        return loss

    def _launch(self, lib, group, ps, gs, ms, vs, ns, step):
        b1, b2 = group['betas']
        numel = (ctypes.c_int64 * len(ns))(*ns)
        _lib.check(lib.dcnr_adam_step(len(ps), _lib.ptr_array(ps), _lib.ptr_array(gs),
                                      _lib.ptr_array(ms), _lib.ptr_array(vs), numel,
                                      float(group['lr']), float(b1), float(b2), float(group['eps']),
                                      float(group['weight_decay']), int(step),
                                      1 if self.decoupled else 0,
                                      _lib.stream_ptr(ps[0].device)), "dcnr_adam_step")


class AdamW(_FusedAdamBase):
    decoupled = True


class Adam(_FusedAdamBase):
    decoupled = False
