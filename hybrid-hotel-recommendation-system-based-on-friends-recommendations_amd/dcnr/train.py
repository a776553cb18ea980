"""Fused training step: the body of the reference's inner loop
(train.py:219-226: zero_grad -> forward -> BCEWithLogits -> backward ->
optimizer.step) as native calls over flat parameter/gradient/moment buffers:

    dcnr_forward(train) -> dcnr_bce_with_logits -> dcnr_backward
      -> [RCCL all-reduce of the flat gradient when data-parallel]
      -> dcnr_adam_step (one launch over every parameter, dense semantics)

Numerically the same update as ``torch.optim.AdamW``/``Adam`` on the
reference's dense gradients (every embedding row's moments decay every step).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib
from .model import DCN_RecSys, run_backward, run_forward
from .ops import bce_with_logits


class FusedTrainer:
    def __init__(self, model: DCN_RecSys, lr=1e-3, weight_decay=1e-2, optimizer_name='AdamW',
                 betas=(0.9, 0.999), eps=1e-8, process_group=None, sync_bn=False):
        if optimizer_name not in ('AdamW', 'Adam'):
            raise ValueError("optimizer_name must be 'AdamW' or 'Adam' (train.py:201-204)")
        self.model = model
        self.flat, self.gflat = model.flatten_()
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.decoupled = optimizer_name == 'AdamW'
        self.step_count = 0
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and
                                                             dist.is_initialized()) else 1
        self._ws = None
        self._grads = [p.grad for p in model.param_tensors()]   # views into gflat
        if sync_bn and self.world > 1:
            from .parallel import install_sync_bn
            install_sync_bn(model, process_group)

    def step(self, user, item, cat, num, y, return_logits=False):
        """One optimisation step on a (local) batch; returns the local loss
        (0-d device tensor) without synchronising the host."""
        model = self.model
        model.train()
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        logits, self._ws = run_forward(model, True, seed, user, item, cat, num, self._ws)
        # grad_scale 1/world: the SUM all-reduce then yields the global mean gradient
        loss, dz = bce_with_logits(logits, y, True, 1.0 / self.world)
        run_backward(model, user, item, cat, num, dz, self._ws, self._grads, seed,
                     accumulate=False)
        if self.world > 1:
            dist.all_reduce(self.gflat, op=dist.ReduceOp.SUM, group=self.pg)
        self.optimizer_step()
        return (loss, logits) if return_logits else loss

    def optimizer_step(self):
        lib = _lib.load()
        self.step_count += 1
        n = (ctypes.c_int64 * 1)(self.flat.numel())
        _lib.check(lib.dcnr_adam_step(1, _lib.ptr_array([self.flat]), _lib.ptr_array([self.gflat]),
                                      _lib.ptr_array([self.m]), _lib.ptr_array([self.v]), n,
                                      float(self.lr), float(self.betas[0]), float(self.betas[1]),
                                      float(self.eps), float(self.wd), self.step_count,
                                      1 if self.decoupled else 0,
                                      _lib.stream_ptr(self.flat.device)), "dcnr_adam_step")
