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

``sparse_reduce_scatter`` is the owner-bucketed sparse exchange of the big
embedding tables' gradients (SURVEY.md 8e option B), used by
``FusedTrainer(exchange="sparse")``: the rows the rank's batch touched
(``touched_rows``: read from the backward's own stable id sort by
``dcnr_emb_touched_rows``, no torch.unique) go to the rank that owns their
ZeRO-1 shard of the flat parameter buffer (one all_to_all of offsets and
rows), and each owner sums what it received in source-rank order into its
gradient shard.  ``sparse_rows_allreduce`` is the earlier host-sized
variant for one table (kept for the CPU tests of the protocol).
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


def sparse_rows_allreduce(grad: torch.Tensor, local_ids: torch.Tensor, group=None) -> dict:
    """Sum a row-sparse embedding gradient over ranks, in place.

    ``grad`` [n_rows, d] holds this rank's dense gradient, nonzero only in
    rows listed in ``local_ids`` (the batch's ids for this table).  Rows are
    owned in contiguous ranges of ceil(n_rows / world).  The exchange:
      1. every rank sends its touched rows (distinct ids, ascending) to their
         owners (all_to_all, sizes exchanged first);
      2. each owner sums what it received in source-rank order (a fixed order:
         every row is summed 0 + g_0 + g_1 + ..., as a single process would);
      3. the owners' summed rows are all-gathered (padded to the largest
         owner list) and written into ``grad``, which is zero elsewhere.
    Every rank ends with the same ``grad``, bit for bit.  Returns the rows
    sent / received counts for reporting."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n, d = grad.shape
    dev = grad.device
    per = (n + world - 1) // world
    uniq = torch.unique(local_ids.reshape(-1))
    rows = grad.index_select(0, uniq)
    send = torch.bincount(torch.div(uniq, per, rounding_mode='floor'), minlength=world)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    sc, rc = send.tolist(), recv.tolist()
    rids = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    dist.all_to_all_single(rids, uniq, rc, sc, group=group)
    rrows = torch.empty((sum(rc), d), dtype=grad.dtype, device=dev)
    dist.all_to_all_single(rrows, rows, rc, sc, group=group)
    lo = rank * per
    span = max(0, min(per, n - lo))
    acc = torch.zeros((span, d), dtype=grad.dtype, device=dev)
    off = 0
    for r in range(world):            # fixed source order; ids distinct per source
        if rc[r]:
            acc.index_add_(0, rids[off:off + rc[r]] - lo, rrows[off:off + rc[r]])
        off += rc[r]
    mine = torch.unique(rids)
    vals = acc.index_select(0, mine - lo)
    cnt = torch.tensor([mine.numel()], dtype=torch.int64, device=dev)
    cnts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    cnts = [int(c.item()) for c in cnts]
    cap = max(max(cnts), 1)
    pid = torch.full((cap,), -1, dtype=torch.int64, device=dev)
    pval = torch.zeros((cap, d), dtype=grad.dtype, device=dev)
    pid[:mine.numel()] = mine
    pval[:mine.numel()] = vals
    aid = torch.empty((world * cap,), dtype=torch.int64, device=dev)
    aval = torch.empty((world * cap, d), dtype=grad.dtype, device=dev)
    dist.all_gather_into_tensor(aid, pid, group=group)
    dist.all_gather_into_tensor(aval, pval, group=group)
    keep = aid >= 0
    grad.zero_()
    grad.index_copy_(0, aid[keep], aval[keep])
    return {"rows_sent": int(uniq.numel()), "rows_owned": int(mine.numel()), "rows_total": sum(cnts)}


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


def sparse_reduce_scatter(gflat: torch.Tensor, gshard: torch.Tensor, width: int,
                          offsets: torch.Tensor, table_counts: torch.Tensor,
                          owner_counts: torch.Tensor, dense_lo: int, dense_hi: int,
                          group=None) -> dict:
    """The reduce-scatter of the embedding segment of ``gflat`` into this
    rank's shard ``gshard`` (ZeRO-1: rank r owns elements [r*Es, (r+1)*Es)),
    moving only touched rows:

      * ``offsets`` [n_tables, B]: per sparse table, this rank's touched rows
        as ascending flat element offsets (row i of table t at
        offsets[t, i] for i < table_counts[t]; each row ``width`` elements,
        never straddling a shard; the tables in flat order);
        ``owner_counts`` [world] how many go to each rank (device tensors,
        as ``touched_rows`` returns them);
      * one all_to_all of the counts, ONE host read of the send / receive /
        table counts, one all_to_all of the offsets and of the rows;
      * the owner zeroes its shard and adds what it received in source-rank
        order (rows distinct per source: the sum is 0 + g_0 + g_1 + ..., the
        same bits for every run);
      * elements [dense_lo, dense_hi) (the small categorical tables) go
        through an all-reduce and their part of the shard is copied in.

    Rows no rank touched have an exactly-zero gradient (the backward
    zero-fills them), so the shard equals the dense reduce-scatter's sum."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    Es = gshard.numel()
    dev = gflat.device
    recv_counts = torch.empty_like(owner_counts)
    dist.all_to_all_single(recv_counts, owner_counts, group=group)
    counts = torch.cat([owner_counts, recv_counts, table_counts]).cpu().tolist()   # one host sync
    sc, rc, tc = counts[:world], counts[world:2 * world], counts[2 * world:]
    send_off = torch.cat([offsets[t, :tc[t]] for t in range(len(tc))])
    col = torch.arange(width, device=dev, dtype=torch.int64)
    rows = gflat[send_off[:, None] + col[None, :]] if send_off.numel() else \
        torch.empty((0, width), dtype=gflat.dtype, device=dev)
    r_off = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    r_rows = torch.empty((sum(rc), width), dtype=gflat.dtype, device=dev)
    dist.all_to_all_single(r_off, send_off, rc, sc, group=group)
    dist.all_to_all_single(r_rows, rows, rc, sc, group=group)
    gshard.zero_()
    gv = gshard.view(-1, width)
    lo = rank * Es
    pos = 0
    for r in range(world):                    # fixed source order
        if rc[r]:
            gv.index_add_(0, torch.div(r_off[pos:pos + rc[r]] - lo, width, rounding_mode="floor"),
                          r_rows[pos:pos + rc[r]])
        pos += rc[r]
    if dense_hi > dense_lo:                   # the small tables: dense all-reduce
        dense = gflat[dense_lo:dense_hi].clone()
        dist.all_reduce(dense, op=dist.ReduceOp.SUM, group=group)
        a, b = max(dense_lo, lo), min(dense_hi, lo + Es)
        if b > a:
            gshard[a - lo:b - lo].copy_(dense[a - dense_lo:b - dense_lo])
    return {"rows_sent": sum(sc), "rows_received": sum(rc),
            "bytes_sent": sum(sc) * (8 + 4 * width) + 4 * max(0, dense_hi - dense_lo)}
