"""Drop-in ``DCN_RecSys`` whose forward/backward run on libdcnr (gfx950 HIP).

Mirrors the reference module (train.py:90-170, duplicated in main.py:61-127):
same constructor signature, same submodules in the same order (so
``torch.manual_seed(s)`` yields the *same* initial weights as the reference),
same ``state_dict`` keys and shapes, same forward signature and
``.squeeze()`` semantics, and ``loss.backward()`` / ``torch.optim`` work
unchanged.  The whole forward (gathers, cross stack, deep tower, head) is one
native call (``dcnr_forward``); the backward is one native call
(``dcnr_backward``).  There is no CPU path: calling forward with CPU tensors
raises.

Extra keywords (not in the reference): ``precision`` -- ``"fp32"`` (default,
f32 MFMA, parity with the reference) or ``"bf16"`` (bf16 MFMA deep tower with
fp32 accumulation and fp32 master weights); ``check_indices`` -- an
out-of-range id raises ``IndexError`` as ``nn.Embedding`` does (train.py:
156-158).  ``True`` (default) checks asynchronously, like the reference on
cuda where the bad index surfaces as a device-side assert at a later
synchronisation: the error is raised by the next call on this model or by
``check_index_errors()``; ``"sync"`` raises in the call itself (a host
synchronisation per call); ``False`` clamps silently.
"""
from __future__ import annotations

import ctypes
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from . import _lib


class CrossLayer(nn.Module):
    """train.py:90-99.  Holds the parameters; the fused path in
    DCN_RecSys.forward never calls this forward (kept for API parity and for
    standalone use): x + x*(x.w) + b."""

    def __init__(self, input_dim):
        super().__init__()
        self.w = nn.Linear(input_dim, 1, bias=False)
        self.b = nn.Parameter(torch.zeros(input_dim))

    def forward(self, x):
        return x + x * self.w(x) + self.b


class ResBlock(nn.Module):
    """train.py:102-122 (parameter container; fused in DCN_RecSys.forward)."""

    def __init__(self, hidden_dim, dropout):
        super().__init__()
        self.layer1 = nn.Linear(hidden_dim, hidden_dim)
        self.bn1 = nn.BatchNorm1d(hidden_dim)
        self.relu = nn.ReLU()
        self.dropout = nn.Dropout(dropout)
        self.layer2 = nn.Linear(hidden_dim, hidden_dim)
        self.bn2 = nn.BatchNorm1d(hidden_dim)

    def forward(self, x):
        identity = x
        out = self.dropout(self.relu(self.bn1(self.layer1(x))))
        out = self.bn2(self.layer2(out))
        out = out + identity
        return self.relu(out)


_PRECISIONS = {"fp32": _lib.PREC_FP32, "bf16": _lib.PREC_BF16}

_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def dropout_seed(dev: torch.device, advance: bool = True) -> int:
    """The 64-bit dropout seed of the next train-mode forward on ``dev``.

    The reference trains on cuda (train.py:32), where ``nn.Dropout`` draws
    from the device's default generator (Philox seed + offset) and leaves the
    CPU generator -- the one ``DataLoader``/``RandomSampler`` draw each
    epoch's permutation from (train.py:195-196) -- untouched.  The seed is
    therefore derived from the device generator's (initial_seed, offset) and
    the offset is advanced, as a Philox launch would: ``torch.manual_seed``
    reproduces the sequence and the CPU generator's stream is not consumed."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    g = torch.cuda.default_generators[idx]
    off = int(g.get_offset())
    if advance:
        g.set_offset(off + 4)
    return _splitmix64((int(g.initial_seed()) & _M64) ^ _splitmix64(off))


class IndexErrorWatch:
    """Deferred id checks: the error word of each call lands in a slot of a
    pinned host ring -- stored there by the forward's last kernel
    (``reserve`` / ``commit``: the slot is the call's ``error_mirror``), or
    copied after the call (``push``) -- stream-ordered, with no event and no
    host wait.  A slot holds PENDING (-1, set by the host before the call)
    until the device's word arrives: 0 = every id in range, else the next
    poll raises IndexError.  Thread-safe: the serving path scores from
    Starlette's threadpool (main.py:306-307 is a sync ``def``), so slot
    assignment and polling hold a lock."""
    RING = 64
    DEPTH = 8      # calls in flight before the oldest is waited for
    PENDING = -1

    SPIN_S = 2e-3  # host spin on one word between queries of its stream

    def __init__(self):
        self.ring = None
        self.pending = []
        self.orphans = []   # slots dropped by a raised error, still PENDING
        self.streams = {}   # slot -> the stream of the call that writes it
        self.free = list(range(self.RING))
        self.lock = threading.Lock()

    def _slot(self):
        if self.ring is None:
            self.ring = torch.zeros(self.RING, dtype=torch.int32, pin_memory=True)
            self.view = self.ring.numpy()   # host view of the pinned words
        self._reclaim()
        if len(self.pending) >= self.DEPTH:
            self._poll(oldest=True)
        if not self.free:
            return None
        slot = self.free.pop(0)
        self.view[slot] = self.PENDING
        return slot

    def reserve(self):
        """A free ring slot and its address (for dcnr_model_desc.error_mirror),
        or (None, None) when every slot is taken."""
        with self.lock:
            slot = self._slot()
        if slot is None:
            return None, None
        return slot, self.ring.data_ptr() + 4 * slot

    def commit(self, slot, stream=None):
        """The call that got ``slot`` is enqueued (on ``stream``): watch its word."""
        with self.lock:
            self.pending.append(slot)
            self.streams[slot] = stream

    def cancel(self, slot):
        with self.lock:
            self.free.append(slot)

    # copies (deepcopy / pickle of the model) start with an empty watch
    def __getstate__(self):
        return {}

    def __setstate__(self, state):
        self.__init__()

    def push(self, word: torch.Tensor):
        """Copy a device error word into a ring slot (stream-ordered)."""
        with self.lock:
            slot = self._slot()
            if slot is not None:
                self.ring[slot:slot + 1].copy_(word.view(torch.int32)[:1], non_blocking=True)
                self.pending.append(slot)
                self.streams[slot] = torch.cuda.current_stream(word.device) \
                    if word.is_cuda else None
                return
        # every slot held by calls still being enqueued: check this one now
        if int(word.view(torch.int32)[0]) != 0:
            raise IndexError("index out of range in self")

    def poll(self, oldest=False, all_=False):
        with self.lock:
            self._poll(oldest, all_)

    def _stream_idle(self, slot):
        """Whether the stream the slot's call was enqueued on has drained.  A
        sticky stream error (a faulting kernel, a launch that failed after
        commit) raises here, as the old per-call event's synchronize did."""
        st = self.streams.get(slot)
        if st is None:
            return False
        return bool(st.query())

    def _wait(self, slot):
        """True once the slot's word has landed; False if its stream drained
        without storing it (the writer never ran)."""
        t0 = time.perf_counter()
        while int(self.view[slot]) == self.PENDING:
            if time.perf_counter() - t0 > self.SPIN_S:
                # the word is late: ask the stream (raises its error, if any)
                if self._stream_idle(slot) and int(self.view[slot]) == self.PENDING:
                    return False
                t0 = time.perf_counter()
            time.sleep(20e-6)
        return True

    def _reclaim(self):
        """Orphaned slots return to the ring once their word has landed, or
        once the stream of the call that owned them has drained without
        storing it (the call never ran to completion: no late store can come;
        ADVICE r05 -- else the 64-slot ring would shrink for good)."""
        if self.orphans:
            left = []
            for s in self.orphans:
                if int(self.view[s]) != self.PENDING:
                    self.free.append(s)
                    continue
                try:
                    idle = self._stream_idle(s)
                except RuntimeError:   # a failed stream stores nothing more either
                    idle = True
                if idle and int(self.view[s]) == self.PENDING:
                    self.view[s] = 0
                    self.free.append(s)
                else:
                    left.append(s)
            self.orphans = left

    def _poll(self, oldest=False, all_=False):
        self._reclaim()
        keep = []
        for n, slot in enumerate(self.pending):
            if all_ or (oldest and n == 0):
                if not self._wait(slot):
                    self.pending = keep + self.pending[n + 1:]
                    self.free.append(slot)
                    raise RuntimeError("id-check word never stored: the call that owned ring "
                                       f"slot {slot} did not run to completion")
            elif int(self.view[slot]) == self.PENDING:
                keep.append(slot)
                continue
            bad = int(self.view[slot]) != 0
            self.free.append(slot)
            if bad:
                # the other words are dropped; a slot whose word has not
                # landed yet is an orphan until it does (_reclaim), so the
                # ring never loses it and a late store never hits a new call
                for sl in keep + self.pending[n + 1:]:
                    if int(self.view[sl]) != self.PENDING:
                        self.free.append(sl)
                    else:
                        self.orphans.append(sl)
                self.pending = []
                raise IndexError("index out of range in self (ids passed to an earlier call)")
        self.pending = keep


class DCN_RecSys(nn.Module):
    """Deep & Cross Network with residual deep tower (train.py:125-170)."""

    def __init__(self, n_users, n_items, cat_dims, n_num_features, params, precision="fp32",
                 check_indices=True):
        super().__init__()
        emb_dim = params['emb_dim']
        hidden_dim = params['hidden_dim']
        n_cross_layers = params['n_cross_layers']
        dropout = params['dropout']
        n_res_blocks = params.get('n_res_blocks', 2)

        self.user_embedding = nn.Embedding(n_users, emb_dim)
        self.item_embedding = nn.Embedding(n_items, emb_dim)
        self.cat_embeddings = nn.ModuleList([
            nn.Embedding(n_cat, int(np.sqrt(n_cat)) + 1) for n_cat in cat_dims.values()])
        cat_emb_sum_dim = sum([int(np.sqrt(n_cat)) + 1 for n_cat in cat_dims.values()])
        input_dim = emb_dim * 2 + cat_emb_sum_dim + n_num_features
        self.initial_deep_layer = nn.Linear(input_dim, hidden_dim)
        self.res_blocks = nn.ModuleList([ResBlock(hidden_dim, dropout) for _ in range(n_res_blocks)])
        self.cross_network = nn.ModuleList([CrossLayer(input_dim) for _ in range(n_cross_layers)])
        final_dim = hidden_dim + input_dim
        self.final_linear = nn.Linear(final_dim, 1)

        if precision not in _PRECISIONS:
            raise ValueError(f"precision must be one of {list(_PRECISIONS)}")
        self.precision = precision
        if check_indices not in (True, False, "sync"):
            raise ValueError("check_indices must be True, False or 'sync'")
        self.check_indices = check_indices
        self._index_watch = IndexErrorWatch()
        self._cat_rows = (ctypes.c_int64 * max(1, len(cat_dims)))(*[int(n) for n in cat_dims.values()])
        self._dims = dict(n_users=n_users, n_items=n_items, cat_dims=list(cat_dims.values()),
                          n_num=n_num_features, emb_dim=emb_dim, hidden=hidden_dim,
                          n_cross=n_cross_layers, n_res=n_res_blocks, dropout=float(dropout),
                          input_dim=input_dim)
        self.keep_intermediates = False   # tests: per-block backward buffers (stage checks)
        self.fused_tower = False   # bf16 eval: fused tower at every batch size (default: B >= 16384)
        self.bn_allreduce = None   # set by dcnr.parallel for SyncBN
        self._sync_bn_hook = None
        self._active_ws = None
        self._flat = None

    # ------------------------------------------------------------ native glue
    def desc(self, grad_ready=None, extra_flags: int = 0) -> _lib.ModelDesc:
        """The native model descriptor.  ``grad_ready``: the backward's
        gradient-group hook (FusedTrainer passes it per call); ``extra_flags``:
        per-call DCNR_FLAG_* (FusedTrainer's DCNR_FLAG_ROW_MAP)."""
        d = self._dims
        desc = _lib.ModelDesc()
        desc.n_users = d['n_users']
        desc.n_items = d['n_items']
        desc.n_cat = len(d['cat_dims'])
        desc.cat_rows = ctypes.cast(self._cat_rows, ctypes.POINTER(ctypes.c_int64))
        desc.emb_dim = d['emb_dim']
        desc.n_num = d['n_num']
        desc.hidden = d['hidden']
        desc.n_cross = d['n_cross']
        desc.n_res = d['n_res']
        desc.dropout = d['dropout']
        desc.precision = _PRECISIONS[self.precision]
        desc.flags = (_lib.FLAG_CHECK_INDICES if self.check_indices else 0) | \
            (_lib.FLAG_KEEP_INTERMEDIATES if getattr(self, 'keep_intermediates', False) else 0) | \
            (_lib.FLAG_FUSED_TOWER if getattr(self, 'fused_tower', False) else 0) | int(extra_flags)
        if self.bn_allreduce is not None:
            desc.bn_allreduce = self.bn_allreduce
        if grad_ready is not None:
            desc.grad_ready = grad_ready
        return desc

    # Host-side dispatch cost matters for small serving batches: building
    # state_dict() per call costs ~150 us, so the (dict, key) slot of every
    # state tensor is resolved once (state_dict order) and the device-pointer
    # table is rebuilt only when a pointer changed (.to(), .data = ...).
    def __setattr__(self, name, value):
        if isinstance(value, nn.Module) and '_slots' in self.__dict__:
            self.__dict__['_slots'] = None
        super().__setattr__(name, value)

    def __getstate__(self):   # pickle / deepcopy: the caches are rebuilt on use
        st = self.__dict__.copy()
        st.pop('_slots', None)
        st.pop('_ptr_cache', None)
        st['_index_watch'] = IndexErrorWatch()
        st.pop('_gc_flag', None)
        st.pop('_cat_rows', None)   # ctypes array: rebuilt by __setstate__
        return st

    def __setstate__(self, st):
        super().__setstate__(st)
        cd = self._dims['cat_dims']
        self.__dict__['_cat_rows'] = (ctypes.c_int64 * max(1, len(cd)))(*[int(n) for n in cd])

    def check_index_errors(self):
        """Wait for every deferred id check of this model; raises IndexError
        if any call saw an out-of-range id."""
        self._index_watch.poll(all_=True)

    def _state_slots(self):
        slots = self.__dict__.get('_slots')
        if slots is None:
            slots = []
            for name in self.state_dict(keep_vars=True).keys():
                path, attr = name.rsplit('.', 1)
                mod = self.get_submodule(path)
                is_p = attr in mod._parameters
                slots.append(((mod._parameters if is_p else mod._buffers), attr, is_p))
            self.__dict__['_slots'] = slots
            self.__dict__['_ptr_cache'] = None
        return slots

    def state_tensors(self) -> List[torch.Tensor]:
        """All state_dict tensors in state_dict order (params + BN buffers)."""
        return [d[k] for d, k, _ in self._state_slots()]

    def param_tensors(self) -> List[torch.Tensor]:
        """named_parameters() order (state_dict order without the buffers)."""
        return [d[k] for d, k, is_p in self._state_slots() if is_p]

    def state_ptr_array(self):
        """ctypes array of the state tensors' device pointers (state_dict order),
        validated (fp32/int64, contiguous) whenever a pointer changed."""
        ts = self.state_tensors()
        key = tuple(t.data_ptr() for t in ts)
        cache = self.__dict__.get('_ptr_cache')
        if cache is not None and cache[0] == key:
            return cache[1]
        for t in ts:
            if t.dtype not in (torch.float32, torch.int64) or not t.is_contiguous():
                raise RuntimeError("dcnr requires fp32 contiguous parameters")
        arr = _lib.ptr_array(ts)
        self.__dict__['_ptr_cache'] = (key, arr)
        return arr

    def workspace_bytes(self, B: int, mode: int, extra_flags: int = 0) -> int:
        lib = _lib.load()
        n = ctypes.c_size_t(0)
        desc = self.desc(extra_flags=extra_flags)
        _lib.check(lib.dcnr_workspace_size(ctypes.byref(desc), int(B), int(mode), ctypes.byref(n)),
                   "dcnr_workspace_size")
        return int(n.value)

    def workspace_offset(self, B: int, mode: int, kind: str, index: int = 0,
                         extra_flags: int = 0) -> int:
        """Byte offset of a stored tensor in the workspace (dcnr_workspace_offset;
        -1 if not materialised)."""
        lib = _lib.load()
        off = ctypes.c_int64(0)
        desc = self.desc(extra_flags=extra_flags)
        _lib.check(lib.dcnr_workspace_offset(ctypes.byref(desc), int(B), int(mode),
                                             _lib.WS_KINDS.index(kind), int(index),
                                             ctypes.byref(off)), "dcnr_workspace_offset")
        return int(off.value)

    def _check_device(self, *tensors):
        dev = self.final_linear.weight.device
        if dev.type != 'cuda':
            raise RuntimeError("dcnr.DCN_RecSys runs on the HIP device only (libdcnr, gfx950); "
                               "move the model to 'cuda' -- there is no CPU path")
        for t in tensors:
            if t.device != dev:
                raise RuntimeError(f"input on {t.device} but model on {dev}")
        return dev

    def prepare_inputs(self, user_ids, item_ids, cat_features, num_features):
        """The forward's inputs as the native call takes them: contiguous
        int64 ids [B], int64 [B, n_cat], fp32 [B, n_num] on the model's
        device (the reference's loop passes column views such as
        ``X_collab_b[:, 0]``, train.py:220)."""
        self._check_device(user_ids, item_ids, cat_features, num_features)
        user_ids = user_ids.reshape(-1).to(torch.int64).contiguous()
        item_ids = item_ids.reshape(-1).to(torch.int64).contiguous()
        B = user_ids.shape[0]
        K, F = len(self._dims['cat_dims']), self._dims['n_num']
        if cat_features.numel() != B * K or num_features.numel() != B * F or \
                item_ids.shape[0] != B:
            raise RuntimeError("input shapes do not match the model")
        cat_features = cat_features.to(torch.int64).reshape(B, K).contiguous()
        num_features = num_features.to(torch.float32).reshape(B, F).contiguous()
        return user_ids, item_ids, cat_features, num_features

    def forward(self, user_ids, item_ids, cat_features, num_features):
        dev = self._check_device(user_ids, item_ids, cat_features, num_features)
        self._index_watch.poll()
        user_ids, item_ids, cat_features, num_features = self.prepare_inputs(
            user_ids, item_ids, cat_features, num_features)
        B = user_ids.shape[0]
        train = self.training
        if train and B == 1:
            raise ValueError("Expected more than 1 value per channel when training, "
                             "got input size torch.Size([1, %d])" % self._dims['hidden'])
        params = self.param_tensors()
        needs_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        seed = dropout_seed(dev) if train else 0
        if needs_grad:
            logits = _DCNRFunction.apply(self, train, seed, user_ids, item_ids, cat_features,
                                         num_features, *params)
        else:
            logits, _ = run_forward(self, train, seed, user_ids, item_ids, cat_features,
                                    num_features)
        return logits.squeeze()

    @torch.no_grad()
    def gather_cross(self, user_ids, item_ids, cat_features, num_features, return_x0=False,
                     out=None):
        """The front of ``forward`` on its own (train.py:156-159, 166-168):
        ``x0 = torch.cat([user_emb, item_emb, *cat_embs, num_features], 1)``
        and ``cross_out`` after the cross network, both fp32 [B, D] (BASELINE
        configs[1]; dcnr_gather_cross).  Returns ``cross_out`` or
        ``(x0, cross_out)``.  ``out``: optional preallocated cross_out.
        With ``check_indices`` an out-of-range id raises IndexError."""
        dev = self._check_device(user_ids, item_ids, cat_features, num_features)
        user_ids = user_ids.reshape(-1).to(torch.int64).contiguous()
        item_ids = item_ids.reshape(-1).to(torch.int64).contiguous()
        B = user_ids.shape[0]
        K, F, D = len(self._dims['cat_dims']), self._dims['n_num'], self._dims['input_dim']
        if cat_features.numel() != B * K or num_features.numel() != B * F or \
                item_ids.shape[0] != B:
            raise RuntimeError("input shapes do not match the model")
        cat_features = cat_features.to(torch.int64).reshape(B, K).contiguous()
        num_features = num_features.to(torch.float32).reshape(B, F).contiguous()
        self._index_watch.poll()
        cross = out if out is not None else torch.empty((B, D), dtype=torch.float32, device=dev)
        if cross.shape != (B, D) or cross.dtype != torch.float32 or not cross.is_contiguous():
            raise ValueError("out must be a contiguous fp32 [B, D] tensor")
        x0 = torch.empty((B, D), dtype=torch.float32, device=dev) if return_x0 else None
        flag = None
        if self.check_indices:   # one error flag per host thread (re-entrant)
            flags = self.__dict__.setdefault('_gc_flag', {})
            key = (threading.get_ident(), dev)
            flag = flags.get(key)
            if flag is None:
                flag = torch.zeros(1, dtype=torch.int32, device=dev)
                flags[key] = flag
            else:
                flag.zero_()
        lib = _lib.load()
        desc = self.desc()
        _lib.check(lib.dcnr_gather_cross(ctypes.byref(desc), self.state_ptr_array(),
                                         user_ids.data_ptr(), item_ids.data_ptr(),
                                         cat_features.data_ptr() if cat_features.numel() else None,
                                         num_features.data_ptr() if num_features.numel() else None,
                                         B, x0.data_ptr() if x0 is not None else None, D,
                                         cross.data_ptr(), D,
                                         flag.data_ptr() if flag is not None else None,
                                         _lib.stream_ptr(dev)), "dcnr_gather_cross")
        if flag is not None:
            if self.check_indices == "sync":
                if int(flag.item()) != 0:
                    raise IndexError("index out of range in self")
            else:
                self._index_watch.push(flag)
        return (x0, cross) if return_x0 else cross

    # ----------------------------------------------------------- flat storage
    def flatten_(self, pad_to: int = 64, table_align: int = 64):
        """Move every parameter into one contiguous fp32 buffer (views keep the
        state_dict API) and give each a ``.grad`` view into one flat gradient
        buffer: lets the fused optimizer and the DP exchange run as single
        launches.  Two segments, each padded to a multiple of ``pad_to`` (the
        optimizer shards split them evenly): the embedding tables
        [0, flat_emb_end) and the dense parameters after them -- the two
        gradient groups dcnr_backward completes one after the other.  Every
        tensor starts on a 64-element boundary; the user and item tables are
        padded to a multiple of ``table_align`` (a multiple of 64: the sparse
        exchange needs their rows on multiples of emb_dim).  Records each
        tensor's element offset in ``flat_offsets``.
        Returns (flat_params, flat_grads)."""
        if table_align % 64:
            raise ValueError("table_align must be a multiple of 64")
        params = self.param_tensors()
        dev = params[0].device
        n_emb = 2 + len(self._dims['cat_dims'])   # the tables lead named_parameters()
        up = lambda x, u: ((x + u - 1) // u) * u   # noqa: E731
        sizes = [up(p.numel(), table_align if k < 2 else 64) for k, p in enumerate(params)]
        emb_end = up(sum(sizes[:n_emb]), pad_to)   # the dense segment starts on a shard boundary
        total = emb_end + up(sum(sizes[n_emb:]), pad_to)
        flat = torch.zeros(total, dtype=torch.float32, device=dev)
        gflat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        offs = []
        for k, (p, sz) in enumerate(zip(params, sizes)):
            if k == n_emb:
                off = emb_end
            n = p.numel()
            offs.append(off)
            flat[off:off + n].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + n].view_as(p)
            p.grad = gflat[off:off + n].view_as(p)
            off += sz
        self._flat = (flat, gflat)
        self.flat_emb_end = emb_end
        self.flat_offsets = offs
        return flat, gflat


def _hook_error(model):
    hook = getattr(model, "_sync_bn_hook", None)
    if hook is not None and hook.error is not None:
        e, hook.error = hook.error, None
        raise RuntimeError("SyncBN all-reduce hook failed") from e


def run_forward(model: DCN_RecSys, train: bool, seed: int, user, item, cat, num,
                ws: Optional[torch.Tensor] = None, extra_flags: int = 0):
    """One native forward.  With ``model.check_indices`` the workspace's
    error word (``ws[:4]``) is checked: in this call (``"sync"``) or through
    the model's deferred watch."""
    lib = _lib.load()
    B = user.shape[0]
    dev = user.device
    mode = _lib.TRAIN if train else _lib.EVAL
    nbytes = model.workspace_bytes(B, mode, extra_flags)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    logits = torch.empty(B, dtype=torch.float32, device=dev)
    state = model.state_ptr_array()
    desc = model.desc(extra_flags=extra_flags)
    # deferred id check: the forward's last kernel stores the error word in a
    # pinned ring slot (no copy on the stream)
    slot = None
    if model.check_indices and model.check_indices != "sync" and B > 0:
        slot, mirror = model._index_watch.reserve()
        if slot is not None:
            desc.error_mirror = mirror
    model._active_ws = ws          # the SyncBN hook (dcnr.parallel) maps pointers into it
    st = lib.dcnr_forward(ctypes.byref(desc), state, user.data_ptr(), item.data_ptr(),
                          cat.data_ptr() if cat.numel() else None,
                          num.data_ptr() if num.numel() else None, B, mode, seed,
                          logits.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev))
    model._active_ws = None
    if slot is not None:
        if st == 0:
            model._index_watch.commit(slot, torch.cuda.current_stream(dev))
        else:
            model._index_watch.cancel(slot)
    _hook_error(model)
    _lib.check(st, "dcnr_forward")
    if model.check_indices == "sync":
        _lib.check(lib.dcnr_check_errors(ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev)),
                   "embedding")
    elif model.check_indices and slot is None and B > 0:
        model._index_watch.push(ws[:4])
    return logits, ws


def run_backward(model: DCN_RecSys, user, item, cat, num, dlogits, ws, grads: List[torch.Tensor],
                 seed: int, accumulate=False, grad_ready=None, extra_flags: int = 0):
    """``seed`` must be the dropout seed of the train-mode forward that filled ws.
    ``grad_ready``: optional dcnr_grad_ready_fn for this call only;
    ``extra_flags``: the forward's per-call flags (the same workspace layout)."""
    lib = _lib.load()
    B = user.shape[0]
    desc = model.desc(grad_ready, extra_flags)
    model._active_ws = ws
    st = lib.dcnr_backward(ctypes.byref(desc), model.state_ptr_array(),
                           _lib.ptr_array(grads), user.data_ptr(), item.data_ptr(),
                           cat.data_ptr() if cat.numel() else None,
                           num.data_ptr() if num.numel() else None, B,
                           dlogits.data_ptr(), int(seed), 1 if accumulate else 0, ws.data_ptr(),
                           ws.numel(), _lib.stream_ptr(user.device))
    model._active_ws = None
    _hook_error(model)
    _lib.check(st, "dcnr_backward")


class _DCNRFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, train, seed, user, item, cat, num, *params):
        logits, ws = run_forward(model, train, seed, user, item, cat, num)
        ctx.model = model
        ctx.train = train
        ctx.seed = seed
        ctx.ws = ws
        ctx.save_for_backward(user, item, cat, num)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        if not ctx.train:
            raise NotImplementedError("dcnr: backward through an eval-mode forward is not "
                                      "supported (call model.train() for training)")
        user, item, cat, num = ctx.saved_tensors
        model = ctx.model
        params = model.param_tensors()
        grads = [torch.empty_like(p) for p in params]
        dl = dlogits.reshape(-1).to(torch.float32).contiguous()
        run_backward(model, user, item, cat, num, dl, ctx.ws, grads, ctx.seed)
        ctx.ws = None
        out = [g if p.requires_grad else None for g, p in zip(grads, params)]
        return (None, None, None, None, None, None, None, *out)
