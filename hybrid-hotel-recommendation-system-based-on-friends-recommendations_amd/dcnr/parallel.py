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

``SparseExchange`` is the owner-bucketed sparse exchange of the big
embedding tables' gradients (SURVEY.md 8e option B), used by
``FusedTrainer(exchange="sparse")``: the rows the rank's batch touched
(``touched_rows``: read from the forward's own stable id sort by
``dcnr_emb_touched_rows``, no torch.unique) go to the rank that owns their
ZeRO-1 shard of the flat parameter buffer (one all_to_all of offsets and
rows), and each owner sums what it received in source-rank order into its
gradient shard.  Both halves are device kernels (``dcnr_sparse_pack`` /
``dcnr_sparse_accumulate``); the message sizes are exchanged right after the
forward and read by the host only after the backward is enqueued, so the
GPU never waits for the host.
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


def touched_rows(model, ws: torch.Tensor, B: int, tables, elem_off, shard_elems: int, world: int):
    """Distinct rows of ``tables`` the batch of the last train-mode forward on
    ``ws`` touched, as flat-buffer element offsets (dcnr_emb_touched_rows):
    returns (offsets [len(tables), B] int64, table_counts [len(tables)],
    owner_counts [world]) on the device; offsets[i, :table_counts[i]] are
    ascending."""
    lib = _lib.load()
    dev = ws.device
    n = len(tables)
    offs = torch.empty((n, max(B, 1)), dtype=torch.int64, device=dev)
    tcnt = torch.empty(n, dtype=torch.int64, device=dev)
    ocnt = torch.empty(world, dtype=torch.int64, device=dev)
    tabs = (ctypes.c_int32 * n)(*[int(t) for t in tables])
    eoff = (ctypes.c_int64 * n)(*[int(o) for o in elem_off])
    desc = model.desc()
    _lib.check(lib.dcnr_emb_touched_rows(ctypes.byref(desc), ws.data_ptr(), ws.numel(), int(B), n,
                                         ctypes.cast(tabs, ctypes.c_void_p),
                                         ctypes.cast(eoff, ctypes.c_void_p), int(shard_elems),
                                         int(world), offs.data_ptr(), tcnt.data_ptr(),
                                         ocnt.data_ptr(), _lib.stream_ptr(dev)),
               "dcnr_emb_touched_rows")
    return offs, tcnt, ocnt


class DeviceSparseOps:
    """The device halves of the sparse exchange (libdcnr).  The CPU tests hand
    SparseExchange a host restatement with the same two methods."""

    def pack(self, grad, offsets, table_counts, width, n_rows):
        """Touched rows (offsets [n_tables, ld], table_counts on the device)
        -> (send offsets [n_rows] int64, send rows [n_rows, width])."""
        lib = _lib.load()
        dev = grad.device
        off = torch.empty(max(n_rows, 1), dtype=torch.int64, device=dev)
        rows = torch.empty((max(n_rows, 1), width), dtype=grad.dtype, device=dev)
        _lib.check(lib.dcnr_sparse_pack(grad.data_ptr(), offsets.data_ptr(), offsets.shape[1],
                                        table_counts.data_ptr(), offsets.shape[0], width,
                                        off.data_ptr(), rows.data_ptr(), _lib.stream_ptr(dev)),
                   "dcnr_sparse_pack")
        return off[:n_rows], rows[:n_rows]

    def accumulate(self, shard, lo, width, offsets, rows, counts):
        """shard = 0 + rows of source 0 + rows of source 1 + ... (counts: host
        list, sources back to back)."""
        lib = _lib.load()
        c = (ctypes.c_int64 * len(counts))(*[int(x) for x in counts])
        _lib.check(lib.dcnr_sparse_accumulate(shard.data_ptr(), int(lo), shard.numel(), width,
                                              offsets.data_ptr() if offsets.numel() else None,
                                              rows.data_ptr() if rows.numel() else None,
                                              ctypes.cast(c, ctypes.c_void_p), len(counts),
                                              _lib.stream_ptr(shard.device)),
                   "dcnr_sparse_accumulate")


_count_streams = {}


class SparseExchange:
    """The reduce-scatter of the embedding segment of the flat gradient into
    this rank's ZeRO-1 shard (rank r owns elements [r*Es, (r+1)*Es)), moving
    only touched rows, in two halves around the backward:

      * ``begin(touched)`` right after the forward: ``touched`` = (offsets
        [n_tables, B], table_counts, owner_counts) as ``touched_rows``
        returns them (the sort that yields them runs under the forward).
        One all_to_all of the owner counts; the send / receive / table
        counts are copied to pinned host memory on a side stream that waits
        for that exchange alone -- not for the backward.
      * ``finish(gflat, gshard)`` after the backward is enqueued: the host
        reads the counts (long since copied), then, stream-ordered after the
        backward: the device pack of the touched rows, the all_to_all of
        offsets and rows, the owner's fixed-order device accumulate (rows
        distinct per source: 0 + g_0 + g_1 + ..., the same bits every run),
        and the all-reduce of elements [dense_lo, dense_hi) (the small
        categorical tables) copied into the shard.

    Only touched rows are read from ``gflat`` and the shard starts from zero,
    so rows no rank touched are exactly zero in it -- the dense
    reduce-scatter's sum -- whether the backward zero-filled the tables or
    wrote only the touched rows (FusedTrainer's row-map step); the
    categorical range must hold the dense gradient (zeroed where untouched)."""

    def __init__(self, width: int, dense_lo: int, dense_hi: int, group=None, ops=None):
        self.width, self.dense_lo, self.dense_hi, self.group = width, dense_lo, dense_hi, group
        self.ops = ops or DeviceSparseOps()
        self._pending = None

    def begin(self, touched):
        offsets, tcnt, ocnt = touched
        world = dist.get_world_size(self.group)
        dev = ocnt.device
        recv = torch.empty_like(ocnt)
        work = dist.all_to_all_single(recv, ocnt, group=self.group, async_op=True)
        n = 2 * world + tcnt.numel()
        if dev.type == "cuda":
            host = torch.empty(n, dtype=torch.int64, pin_memory=True)
            side = _count_streams.get(dev)
            if side is None:
                side = _count_streams[dev] = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))   # the counts' producers
            with torch.cuda.stream(side):
                work.wait()                                     # ... and the exchange, nothing later
                host.copy_(torch.cat([ocnt, recv, tcnt]), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
        else:
            work.wait()
            host, ev = torch.cat([ocnt, recv, tcnt]), None
        self._pending = (offsets, tcnt, ocnt, recv, host, ev)

    def finish(self, gflat: torch.Tensor, gshard: torch.Tensor) -> dict:
        offsets, tcnt, ocnt, recv, host, ev = self._pending
        self._pending = None
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        if ev is not None:
            ev.synchronize()
        counts = host.tolist()
        sc, rc = counts[:world], counts[world:2 * world]
        width, Es = self.width, gshard.numel()
        dev = gflat.device
        send_off, rows = self.ops.pack(gflat, offsets, tcnt, width, sum(sc))
        r_off = torch.empty(sum(rc), dtype=torch.int64, device=dev)
        r_rows = torch.empty((sum(rc), width), dtype=gflat.dtype, device=dev)
        dist.all_to_all_single(r_off, send_off, rc, sc, group=self.group)
        dist.all_to_all_single(r_rows, rows, rc, sc, group=self.group)
        lo = rank * Es
        self.ops.accumulate(gshard, lo, width, r_off, r_rows, rc)
        dense_lo, dense_hi = self.dense_lo, self.dense_hi
        if dense_hi > dense_lo:                   # the small tables: dense all-reduce
            dense = gflat[dense_lo:dense_hi].clone()
            dist.all_reduce(dense, op=dist.ReduceOp.SUM, group=self.group)
            a, b = max(dense_lo, lo), min(dense_hi, lo + Es)
            if b > a:
                gshard[a - lo:b - lo].copy_(dense[a - dense_lo:b - dense_lo])
        return {"rows_sent": sum(sc), "rows_received": sum(rc),
                "bytes_sent": sum(sc) * (8 + 4 * width) + 4 * max(0, dense_hi - dense_lo)}
