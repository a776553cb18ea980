"""Data-parallel plumbing for the DCN-R hot path (one process per GPU).

The reference trains in one process (train.py:195-240); scaling it out is a
plain data-parallel split of each batch across ranks:

  * ``shard_range`` -- rank r owns rows [lo, hi) of a global batch (the
    contiguous split a DistributedSampler with drop_last would give).
  * the gradient exchange is ONE all-reduce of the flat fp32 gradient buffer
    (``FusedTrainer.step``; RCCL over xGMI on the GPU box, gloo in CPU tests),
    with the BCE gradient pre-scaled by 1/world so the SUM is the global mean.
  * optional SyncBN: ``install_sync_bn`` registers a ``dcnr_allreduce_fn``
    hook.  libdcnr then hands every BatchNorm's fp64 statistics buffer
    [sum t | sum t^2 | (unused) | count] (forward) and [sum dy | sum dy*xhat |
    sum dz*out | count] (backward) to the hook, which sums it over ranks in
    place before the finalize kernel runs -- normalisation then uses the
    global batch's mean/var exactly as one big batch would.

Default (sync_bn=False) is local BN: every rank normalises with its own
batch, like torch DDP without SyncBatchNorm.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib


def shard_range(n: int, rank: int, world: int):
    """Contiguous, equal split of n rows (the last ``n % world`` rows are
    dropped so every rank sees the same local batch, as the bench needs)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    per = n // world
    return rank * per, (rank + 1) * per


class SyncBNHook:
    """Callable matching ``dcnr_allreduce_fn``.  The device buffer always lies
    inside the workspace tensor of the native call in flight, which the model
    publishes as ``model._active_ws`` just before the call; the hook turns the
    raw pointer back into a float64 view of that tensor and all-reduces it on
    the current stream (the stream libdcnr launches on)."""

    def __init__(self, model, group=None):
        self.model = model
        self.group = group
        self.calls = 0
        self.error: Optional[BaseException] = None
        self.cfunc = _lib.ALLREDUCE_FN(self._cb)

    def buffer_view(self, ptr: int, count: int) -> torch.Tensor:
        ws = getattr(self.model, "_active_ws", None)
        if ws is None:
            raise RuntimeError("SyncBN hook called outside a dcnr call")
        off = ptr - ws.data_ptr()
        nbytes = count * 8
        if off < 0 or off + nbytes > ws.numel() or off % 8:
            raise RuntimeError("SyncBN buffer not inside the active workspace")
        return ws[off:off + nbytes].view(torch.float64)

    def __call__(self, ptr: int, count: int):
        buf = self.buffer_view(ptr, count)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
        self.calls += 1

    def _cb(self, ctx, ptr, count, stream):
        try:
            self(int(ptr), int(count))
            return 0
        except BaseException as e:  # never unwind through the C ABI
            self.error = e
            return 1


def install_sync_bn(model, group=None) -> SyncBNHook:
    hook = SyncBNHook(model, group)
    model._sync_bn_hook = hook          # keeps the ctypes thunk alive
    model.bn_allreduce = hook.cfunc
    return hook


def remove_sync_bn(model):
    model.bn_allreduce = None
    model._sync_bn_hook = None
