"""Fused training step: the body of the reference's inner loop
(train.py:219-226: zero_grad -> forward -> BCEWithLogits -> backward ->
optimizer.step) as native calls over flat parameter/gradient/moment buffers:

    dcnr_forward(train) -> dcnr_bce_with_logits -> dcnr_backward
      -> data-parallel exchange + dcnr_adam_step (dense semantics):
         world == 1: one launch over every parameter
         world > 1: the flat buffers have two segments (model.flatten_): the
           embedding tables (~95 % of the bytes) and the dense parameters.
           dcnr_backward completes the dense group first (its
           DCNR_GRADS_DENSE hook fires before the dx0 GEMM and the whole
           embedding backward), and the hook starts the dense segment's
           all-reduce right there, so it runs under the embedding backward.
           Then the embedding segment:
           shard_optimizer (default): reduce-scatter (RCCL), AdamW on this
             rank's 1/world shard with its 1/world of the moments,
             all-gather of the updated parameters -- the all-reduce's bytes,
             1/world of the optimizer's HBM traffic and moment memory
             (ZeRO-1 style); the dense segment is updated whole on every rank,
             under the first reduce-scatter.  The segment is exchanged in
             ``exchange_chunks`` pieces (default 4), each split over the ranks,
             so a rank owns one piece of every chunk and each chunk's
             reduce-scatter input and all-gather output are contiguous; the
             chunks run as a pipeline over two communicators (two RCCL
             streams): reduce-scatter(c+1) under AdamW(c) under
             all-gather(c-1), the segment's tail (the item and categorical
             tables) first
           shard_optimizer=False: all-reduce, every rank updates everything
           exchange="sparse" (ZeRO-1 like the default): the user and item
             tables' gradient rows the rank's batch touched -- read from the
             forward's own id sort (dcnr_emb_touched_rows) -- go to the
             owners of their parameter shard (all_to_all), each owner sums
             them in rank order into its shard (dcnr.parallel.SparseExchange:
             device pack and accumulate; the message sizes are exchanged
             after the forward and read once the backward is enqueued, so the
             GPU never idles for the host), the small categorical tables go
             through an all-reduce; then AdamW on the shard and the
             all-gather of the parameters, as above

Numerically the same update as ``torch.optim.AdamW``/``Adam`` on the
reference's dense gradients (every embedding row's moments decay every step).

world == 1 (unless ``dense_table_grads=True``): the backward does not zero the
tables' gradients (142 MB at the bench shape) but marks the rows it writes in a
byte map (DCNR_FLAG_ROW_MAP), and the optimizer launch reads unmarked rows'
gradients as exactly 0 (dcnr_adam_step_rows): the same parameters bit for bit,
without the zero fill and without reading the untouched rows' gradients.  The
tables' ``.grad`` rows a step did not touch then hold stale values: call
``FusedTrainer.materialize_table_grads()`` before reading them (gradient-norm
logging, ``clip_grad_norm_``), or pass ``dense_table_grads=True``.
world > 1 with exchange="sparse" (same opt-out): the same backward, since the
exchange reads only the touched rows of the user and item tables; the small
categorical tables, all-reduced densely, are zeroed before it.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib
from .model import DCN_RecSys, dropout_seed, run_backward, run_forward
from .ops import bce_with_logits


class FusedTrainer:
    """The reference's training step (train.py:219-226) as native calls; see
    the module docstring.  ``dense_table_grads=False`` (default) at world 1
    leaves the tables' untouched ``.grad`` rows stale after ``step()`` --
    ``materialize_table_grads()`` zeroes them when a caller reads them."""

    def __init__(self, model: DCN_RecSys, lr=1e-3, weight_decay=1e-2, optimizer_name='AdamW',
                 betas=(0.9, 0.999), eps=1e-8, process_group=None, sync_bn=False,
                 shard_optimizer=None, exchange="dense", sparse_ops=None, dense_table_grads=False,
                 exchange_chunks=4):
        if optimizer_name not in ('AdamW', 'Adam'):
            raise ValueError("optimizer_name must be 'AdamW' or 'Adam' (train.py:201-204)")
        self.model = model
        self.pg = process_group
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if dist_on else 1
        self.rank = dist.get_rank(process_group) if dist_on else 0
        if exchange not in ("dense", "sparse"):
            raise ValueError("exchange must be 'dense' or 'sparse'")
        self.exchange = exchange
        if exchange == "sparse":
            if shard_optimizer is False:
                raise ValueError("exchange='sparse' reduce-scatters into optimizer shards: "
                                 "it needs shard_optimizer=True (or None)")
            if self.world > _lib.TOUCHED_MAX_WORLD:
                raise ValueError(f"exchange='sparse' supports at most {_lib.TOUCHED_MAX_WORLD} "
                                 f"ranks (world {self.world})")
            shard_optimizer = True
        self.shard = (self.world > 1) if shard_optimizer is None else bool(shard_optimizer)
        if int(exchange_chunks) < 1:
            raise ValueError("exchange_chunks must be >= 1")
        # the dense exchange's pipeline depth (module docstring); the sparse
        # exchange keeps one contiguous shard per rank (its owners are offset // Es)
        self.chunks = int(exchange_chunks) if (self.shard and exchange == "dense"
                                               and self.world > 1) else 1
        # the pipeline's all-gathers run on a second communicator (its own
        # stream), beside the reduce-scatters on the first
        self._ag_pg = None
        if self.chunks > 1:
            ranks = (dist.get_process_group_ranks(process_group) if process_group is not None
                     else list(range(self.world)))
            self._ag_pg = dist.new_group(ranks=ranks, use_local_synchronization=True)
        # the sparse exchange's layout: the user and item tables at flat
        # offsets 0 and nu (rows of emb_dim elements), the categorical tables
        # after them (dense all-reduce); rows must not straddle a shard, so
        # both tables and the shards are padded to multiples of lcm(64, emb_dim)
        d = model._dims['emb_dim']
        unit = 64 * d // math.gcd(64, d) if exchange == "sparse" else 64
        self.flat, self.gflat = model.flatten_(pad_to=unit * self.world * self.chunks,
                                               table_align=unit)
        self.E = model.flat_emb_end                      # embedding segment [0, E)
        N = self.flat.numel()
        self.Es = self.E // self.world if self.shard else self.E   # this rank's embedding moments
        offs = model.flat_offsets
        self._sparse_layout = dict(width=d, tables=(0, 1), elem_off=(offs[0], offs[1]),
                                   dense_lo=offs[2], dense_hi=self.E)
        self._sparse_ok = self.shard and not (self.Es % d or offs[1] % d)
        if exchange == "sparse" and not self._sparse_ok:   # (cannot happen with the padding above)
            raise ValueError("exchange='sparse' needs table rows aligned to the optimizer "
                             f"shards (emb_dim {d}, shard {self.Es} elements)")
        self._B = 0
        self.last_exchange = None
        self._sparse = None
        if self._sparse_ok and self.world > 1:
            from .parallel import SparseExchange
            lay = self._sparse_layout
            self._sparse = SparseExchange(d, lay["dense_lo"], lay["dense_hi"], process_group,
                                          ops=sparse_ops)
        self.m = torch.zeros(self.Es + N - self.E, dtype=torch.float32, device=self.flat.device)
        self.v = torch.zeros_like(self.m)
        self.gshard = torch.empty(self.Es, dtype=torch.float32,
                                  device=self.flat.device) if self.shard else None
        self._dense_work = None
        self._hook_error = None
        # world > 1: the dense segment's all-reduce starts from inside the
        # backward.  The hook is handed to this trainer's own dcnr_backward
        # calls only (run_backward(grad_ready=...)), never installed on the
        # model: a plain autograd backward must not start an exchange.
        self._grad_ready_cb = _lib.GRAD_READY_FN(self._on_grads_ready) if self.world > 1 else None
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.decoupled = optimizer_name == 'AdamW'
        self.step_count = 0
        self._ws = None
        self._grads = [p.grad for p in model.param_tensors()]   # views into gflat
        # world 1: the row-map step (module docstring)
        self.row_map = self.world == 1 and not dense_table_grads
        self.dense_table_grads = dense_table_grads
        self._flags = _lib.FLAG_ROW_MAP if self.row_map else 0
        self._rows_cache = None
        # a list: step() appends (backward end, step end) CUDA events to it
        self.step_events = None
        if sync_bn and self.world > 1:
            from .parallel import install_sync_bn
            install_sync_bn(model, process_group)

    def step(self, user, item, cat, num, y, return_logits=False):
        """One optimisation step on a (local) batch; returns the local loss
        (0-d device tensor) without synchronising the host."""
        model = self.model
        model.train()
        user, item, cat, num = model.prepare_inputs(user, item, cat, num)
        y = y.reshape(-1).to(torch.float32).contiguous()
        seed = dropout_seed(user.device)
        model._index_watch.poll()
        sparse_rows = self._sparse_rows()
        flags = self._flags | (_lib.FLAG_ROW_MAP if sparse_rows else 0)
        logits, self._ws = run_forward(model, True, seed, user, item, cat, num, self._ws,
                                       extra_flags=flags)
        self._B = user.shape[0]
        if self.exchange == "sparse" and self._sparse is not None:
            # the touched rows come from the forward's id sort: their counts
            # are exchanged now, under the backward
            self._sparse.begin(self.touched_rows())
        # grad_scale 1/world: the SUM all-reduce then yields the global mean gradient
        loss, dz = bce_with_logits(logits, y, True, 1.0 / self.world)
        self._dense_work = None
        if sparse_rows:
            # the categorical tables go through a dense all-reduce: zero them
            # (1.5 MB at the bench shape); the row map leaves their untouched
            # rows unwritten
            lay = self._sparse_layout
            self.gflat[lay["dense_lo"]:lay["dense_hi"]].zero_()
        try:
            run_backward(model, user, item, cat, num, dz, self._ws, self._grads, seed,
                         accumulate=False, grad_ready=self._grad_ready_cb,
                         extra_flags=flags)
        except RuntimeError:
            # the hook may have started the dense all-reduce before the
            # failure: let it finish before anyone writes gflat again
            work, self._dense_work = self._dense_work, None
            if work is not None:
                try:
                    work.wait()
                except Exception:   # noqa: BLE001 -- the original error is what matters
                    pass
            if self._hook_error is not None:
                err, self._hook_error = self._hook_error, None
                raise RuntimeError("gradient exchange hook failed") from err
            raise
        # the all-reduce this step's backward started (None: start it now)
        dense, self._dense_work = self._dense_work, None
        marks = self.step_events
        if marks is not None:   # the backward's last kernel is enqueued
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.row_map:
            self.step_count += 1
            self._adam_rows(self.step_count)
        else:
            self._exchange_and_update(None, None, dense)
        if marks is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            marks.append((e0, e1))
        return (loss, logits) if return_logits else loss

    def materialize_table_grads(self):
        """Zero the table-gradient rows the last row-map step did not write.

        With the row map (world 1 by default, and the sparse exchange) the
        backward leaves an untouched row's ``.grad`` as it was, where the
        reference's ``zero_grad()`` + ``backward()`` (train.py:222-225) leaves
        it 0: code that reads the tables' ``p.grad`` after ``step()``
        (gradient-norm logging, ``clip_grad_norm_``) calls this first.  The
        parameters and moments do not depend on it (dcnr_adam_step_rows reads
        an unmarked row as 0).  No-op without the row map."""
        if self._ws is None or not (self.row_map or self._sparse_rows()):
            return
        model = self.model
        map_off = model.workspace_offset(self._B, _lib.TRAIN, "row_map", extra_flags=_lib.FLAG_ROW_MAP)
        if map_off < 0:
            raise RuntimeError("train workspace has no row map")
        d = model._dims
        rows = [d['n_users'], d['n_items']] + list(d['cat_dims'])
        kb = 0
        for t, r in enumerate(rows):
            untouched = self._ws[map_off + kb:map_off + kb + r] == 0
            self._grads[t][untouched] = 0.0
            kb += r

    def exchange_window_ms(self):
        """Mean time between the end of the backward and the end of the step
        (exchange + optimizer: what the step adds after its last backward
        kernel) over the steps recorded since ``step_events = []``."""
        marks = self.step_events or []
        if not marks:
            return None
        marks[-1][1].synchronize()
        return sum(a.elapsed_time(b) for a, b in marks) / len(marks)

    def _sparse_rows(self):
        """world > 1 with the sparse exchange: the backward writes only the
        rows the batch touched (DCNR_FLAG_ROW_MAP, no 142 MB zero fill); the
        exchange packs exactly those rows, and the owner's accumulate starts
        its shard from zero, so the shard is the same sum bit for bit."""
        return (self.world > 1 and self.exchange == "sparse" and self._sparse is not None
                and not self.dense_table_grads)

    def _row_segments(self):
        """dcnr_adam_step_rows' tensor list over the flat buffers: each table
        with its slice of the workspace's row map, the gaps and the dense
        segment without (cached per workspace pointer and batch)."""
        ws, B = self._ws, self._B
        key = (ws.data_ptr(), B)
        if self._rows_cache is not None and self._rows_cache[0] == key:
            return self._rows_cache[1]
        model = self.model
        map_off = model.workspace_offset(B, _lib.TRAIN, "row_map", extra_flags=_lib.FLAG_ROW_MAP)
        if map_off < 0:
            raise RuntimeError("train workspace has no row map")
        d = model._dims
        rows = [d['n_users'], d['n_items']] + list(d['cat_dims'])
        offs = model.flat_offsets
        params = model.param_tensors()
        segs = []   # (lo, numel, map pointer or None, width)
        pos, kb = 0, 0
        for t, r in enumerate(rows):
            if offs[t] > pos:
                segs.append((pos, offs[t] - pos, None, 1))
            w = params[t].shape[1]
            segs.append((offs[t], r * w, ws.data_ptr() + map_off + kb, w))
            pos, kb = offs[t] + r * w, kb + r
        N = self.flat.numel()
        if N > pos:
            segs.append((pos, N - pos, None, 1))
        n = len(segs)
        P = lambda buf: (ctypes.c_void_p * n)(*[buf.data_ptr() + 4 * lo for lo, *_ in segs])  # noqa: E731
        arrs = (P(self.flat), P(self.gflat), P(self.m), P(self.v),
                (ctypes.c_int64 * n)(*[c for _, c, _, _ in segs]),
                (ctypes.c_void_p * n)(*[mp for _, _, mp, _ in segs]),
                (ctypes.c_int32 * n)(*[w for _, _, _, w in segs]), n)
        self._rows_cache = (key, arrs)
        return arrs

    def _adam_rows(self, step):
        """The world-1 optimizer step of a row-map backward (module docstring)."""
        p, g, m, v, numel, maps, widths, n = self._row_segments()
        lib = _lib.load()
        _lib.check(lib.dcnr_adam_step_rows(n, p, g, m, v, numel, maps, widths,
                                           float(self.lr), float(self.betas[0]),
                                           float(self.betas[1]), float(self.eps), float(self.wd),
                                           int(step), 1 if self.decoupled else 0,
                                           _lib.stream_ptr(self.flat.device)),
                   "dcnr_adam_step_rows")

    def _on_grads_ready(self, ctx, group, stream):
        """dcnr_grad_ready_fn: the dense gradients are enqueued -> start their
        all-reduce now (ordered after the stream's work so far)."""
        try:
            if group == _lib.GRADS_DENSE:
                self._dense_work = dist.all_reduce(self.gflat[self.E:], op=dist.ReduceOp.SUM,
                                                   group=self.pg, async_op=True)
            return 0
        except Exception as e:   # noqa: BLE001 -- reported after the C call returns
            self._hook_error = e
            return 1

    def check_indices(self):
        """Wait for every step's id check; raises IndexError if any failed
        (the checks are otherwise reported by a later step)."""
        self.model.check_index_errors()

    def exchange_and_update(self, adam=None, touched=None):
        """The data-parallel gradient exchange and the optimizer step on the
        flat buffers.  ``adam(p, g, m, v, step)`` defaults to dcnr_adam_step
        (the CPU tests pass a host restatement to check the exchange).
        ``touched``: for the sparse exchange, (offsets, table_counts,
        owner_counts) as dcnr.parallel.touched_rows returns them (default:
        read from the last step's backward)."""
        self._exchange_and_update(adam, touched, None)

    def touched_rows(self):
        """The rows the last step's batch touched in the sparse-exchanged
        tables (dcnr_emb_touched_rows over the step's workspace)."""
        from .parallel import touched_rows
        lay = self._sparse_layout
        return touched_rows(self.model, self._ws, self._B, lay["tables"], lay["elem_off"], self.Es,
                            self.world)

    def _exchange_and_update(self, adam, touched, dense):
        adam = adam or self._adam
        self.step_count += 1
        E, Es, world = self.E, self.Es, self.world
        if world == 1:
            adam(self.flat, self.gflat, self.m, self.v, self.step_count)
            return
        if dense is None:   # not started by this step's backward: start it now
            dense = dist.all_reduce(self.gflat[E:], op=dist.ReduceOp.SUM, group=self.pg,
                                    async_op=True)
        if self.shard:
            if self.exchange == "sparse":
                if self._sparse is None:
                    raise ValueError("exchange='sparse': table rows not aligned to the shards")
                if touched is not None or self._sparse._pending is None:
                    self._sparse.begin(touched if touched is not None else self.touched_rows())
                self.last_exchange = self._sparse.finish(self.gflat, self.gshard)
                pshard = self.flat[self.rank * Es:(self.rank + 1) * Es]
                adam(pshard, self.gshard, self.m[:Es], self.v[:Es], self.step_count)
                dist.all_gather_into_tensor(self.flat[:E], pshard, group=self.pg)
            else:
                dense = self._chunked_exchange(adam, dense)
        else:
            dist.all_reduce(self.gflat[:E], op=dist.ReduceOp.SUM, group=self.pg)
            adam(self.flat[:E], self.gflat[:E], self.m[:E], self.v[:E], self.step_count)
        if dense is not None:
            dense.wait()
            adam(self.flat[E:], self.gflat[E:], self.m[Es:], self.v[Es:], self.step_count)

    def shard_ranges(self):
        """The flat ranges [lo, hi) of the embedding segment this rank owns,
        in the order its ``gshard`` and embedding moments hold them (one range
        unless the dense exchange runs in chunks; empty without sharding).
        The sparse exchange owns one contiguous range per rank, so switching
        ``exchange`` on a live trainer with chunks > 1 re-assigns the
        embedding moments (bench.py does it only to time the other exchange)."""
        if not self.shard:
            return []
        W, r, C = self.world, self.rank, self.chunks
        if self.exchange == "sparse":
            return [(r * self.Es, (r + 1) * self.Es)]
        cs = self.Es // C
        return [(c * W * cs + r * cs, c * W * cs + (r + 1) * cs) for c in range(C)]

    def _chunked_exchange(self, adam, dense):
        """The dense embedding exchange as a pipeline of ``self.chunks``
        chunks (module docstring).  Chunk c is the flat range
        [c W cs, (c+1) W cs) (cs = Es / chunks, W = world); rank r owns its
        piece [c W cs + r cs, c W cs + (r+1) cs), whose gradient and moments
        are gshard / m / v [c cs, (c+1) cs).  The communicator runs its
        collectives in issue order: every reduce-scatter is issued up front on
        the trainer's group, each all-gather on a second group (its own
        stream) once its chunk's AdamW is enqueued, so RS(c+1) runs under
        AdamW(c) and beside AG(c-1).  Each element is still the SUM of the ranks'
        gradients (at world 2 the same bits as one reduce-scatter).  Returns
        None once the dense segment's AdamW is enqueued."""
        E, Es, W, r, C = self.E, self.Es, self.world, self.rank, self.chunks
        cs = Es // C
        order = list(range(C))[::-1]   # the segment's tail (item, categorical tables) first
        rs = {c: dist.reduce_scatter_tensor(self.gshard[c * cs:(c + 1) * cs],
                                            self.gflat[c * W * cs:(c + 1) * W * cs],
                                            op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
              for c in order}
        # the dense segment's AdamW (its all-reduce ran under the embedding
        # backward) goes under the first reduce-scatters
        dense.wait()
        adam(self.flat[E:], self.gflat[E:], self.m[Es:], self.v[Es:], self.step_count)
        gathers = []
        for c in order:
            rs.pop(c).wait()
            lo = c * W * cs + r * cs
            pc = self.flat[lo:lo + cs]
            adam(pc, self.gshard[c * cs:(c + 1) * cs], self.m[c * cs:(c + 1) * cs],
                 self.v[c * cs:(c + 1) * cs], self.step_count)
            gathers.append(dist.all_gather_into_tensor(self.flat[c * W * cs:(c + 1) * W * cs], pc,
                                                       group=self._ag_pg, async_op=True))
        for g in gathers:
            g.wait()
        return None

    def optimizer_step(self):
        """Adam/AdamW over the local flat gradient (no exchange)."""
        if self.shard:
            raise RuntimeError("optimizer_step: the moments are sharded; use exchange_and_update")
        self.step_count += 1
        self._adam(self.flat, self.gflat, self.m, self.v, self.step_count)

    def _adam(self, p, g, m, v, step):
        lib = _lib.load()
        n = (ctypes.c_int64 * 1)(p.numel())
        _lib.check(lib.dcnr_adam_step(1, _lib.ptr_array([p]), _lib.ptr_array([g]),
                                      _lib.ptr_array([m]), _lib.ptr_array([v]), n,
                                      float(self.lr), float(self.betas[0]), float(self.betas[1]),
                                      float(self.eps), float(self.wd), int(step),
                                      1 if self.decoupled else 0,
                                      _lib.stream_ptr(p.device)), "dcnr_adam_step")
