"""Cosine nearest neighbours on libdcnr: drop-in for the
``sklearn.neighbors.NearestNeighbors(metric='cosine', algorithm='brute')``
index the reference builds at startup (main.py:268-270) and queries per
positive hotel (main.py:200) and per /similar_items request (main.py:300).

``kneighbors`` keeps sklearn's contract (numpy in, numpy ``(dist, idx)`` out,
ascending distance, the query row itself included when it is in the index --
callers drop position 0 as main.py does).  Ties are ordered by row index
(sklearn's argsort order among exactly equal distances is unspecified).
``kneighbors_device`` takes/returns device tensors for batched callers.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

# the batched scan (knn.hip scan v4) serves d = 32 / 64 over tables larger
# than its 32768-row sample; only those get the fit-time bf16 copy
PACKED_D = (32, 64)
PACKED_MIN_ROWS = 32768


class NearestNeighbors:
    def __init__(self, n_neighbors=5, metric='cosine', algorithm='brute', device='cuda'):
        if metric != 'cosine':
            raise NotImplementedError("dcnr.NearestNeighbors implements metric='cosine' only "
                                      "(the reference's only use, main.py:268)")
        if algorithm not in ('brute', 'auto'):
            raise NotImplementedError("dcnr.NearestNeighbors is a brute-force index")
        self.n_neighbors = n_neighbors
        self.metric = metric
        self.algorithm = algorithm
        self.device = torch.device(device)
        self._table = None
        self._inv = None
        self._packed = None

    def fit(self, X, y=None):
        t = torch.as_tensor(np.asarray(X, dtype=np.float32) if not torch.is_tensor(X) else X)
        t = t.to(self.device, torch.float32).contiguous()
        if t.dim() != 2:
            raise ValueError("Expected 2D array")
        if self.device.type != 'cuda':
            raise RuntimeError("dcnr.NearestNeighbors runs on the HIP device only")
        self._table = t
        self._inv = torch.empty(t.shape[0], dtype=torch.float32, device=self.device)
        lib = _lib.load()
        _lib.check(lib.dcnr_row_inv_norms(t.data_ptr(), t.shape[0], t.shape[1], self._inv.data_ptr(),
                                          _lib.stream_ptr(self.device)), "dcnr_row_inv_norms")
        self._packed = None
        if t.shape[1] in PACKED_D and t.shape[0] > PACKED_MIN_ROWS:
            # bf16 copy of the normalised rows for the batched coarse scan
            # (2 B / element beside the fp32 table; same results without it)
            self._packed = torch.empty(t.shape, dtype=torch.int16, device=self.device)
            _lib.check(lib.dcnr_cosine_pack_rows(t.data_ptr(), self._inv.data_ptr(), t.shape[0],
                                                 t.shape[1], self._packed.data_ptr(),
                                                 _lib.stream_ptr(self.device)),
                       "dcnr_cosine_pack_rows")
        self.n_samples_fit_ = t.shape[0]
        self.n_features_in_ = t.shape[1]
        return self

    def kneighbors_device(self, q: torch.Tensor, k: int):
        if self._table is None:
            raise RuntimeError("This NearestNeighbors instance is not fitted yet")
        lib = _lib.load()
        q = q.to(self.device, torch.float32).reshape(-1, self._table.shape[1]).contiguous()
        Q = q.shape[0]
        N, d = self._table.shape
        if k > N:
            raise ValueError(f"Expected n_neighbors <= n_samples_fit, but n_neighbors = {k}, "
                             f"n_samples_fit = {N}, n_samples = {Q}")
        idx = torch.empty((Q, k), dtype=torch.int64, device=self.device)
        dist = torch.empty((Q, k), dtype=torch.float32, device=self.device)
        nb = int(lib.dcnr_cosine_topk_workspace_size(N, Q, k))
        ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=self.device)
        packed = self._packed.data_ptr() if self._packed is not None else None
        _lib.check(lib.dcnr_cosine_topk_packed(self._table.data_ptr(), self._inv.data_ptr(), packed,
                                               N, d, q.data_ptr(), Q, k, idx.data_ptr(),
                                               dist.data_ptr(), ws.data_ptr(), ws.numel(),
                                               _lib.stream_ptr(self.device)),
                   "dcnr_cosine_topk")
        return dist, idx

    def kneighbors(self, X=None, n_neighbors=None, return_distance=True):
        k = self.n_neighbors if n_neighbors is None else int(n_neighbors)
        if k <= 0:
            raise ValueError(f"Expected n_neighbors > 0. Got {k}")
        q = torch.as_tensor(np.asarray(X, dtype=np.float32)) if not torch.is_tensor(X) else X
        if q.shape[0] == 0:   # sklearn's check_array
            raise ValueError(f"Found array with 0 sample(s) (shape={tuple(q.shape)}) while a minimum "
                             "of 1 is required by NearestNeighbors.")
        dist, idx = self.kneighbors_device(q, k)
        idx_np = idx.cpu().numpy()
        if return_distance:
            return dist.cpu().numpy(), idx_np
        return idx_np


def index_shard(n: int, rank: int, world: int):
    """Rows [lo, hi) of an n-row index held by ``rank``: balanced, covering
    every row (unlike parallel.shard_range, which trims a batch)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return n * rank // world, n * (rank + 1) // world


class ShardedNearestNeighbors:
    """The cosine index row-sharded over a process group (SURVEY.md 8(e),
    cfg5): rank r holds rows ``index_shard(N, r, world)`` of the table, scans
    only those (``dcnr_cosine_topk``), and the ranks' k-lists -- global row
    ids -- are all-gathered (world * Q * k candidates, one exchange step) and
    merged on the device by ``dcnr_topk_merge``.  Every rank returns exactly
    what ``NearestNeighbors`` over the whole table returns, ties included
    (ascending (dist, row)); the per-row distance does not depend on which
    rank computes it.  Same ``kneighbors`` contract as the single index
    (main.py:200, 300); every rank must call with the same queries."""

    def __init__(self, n_neighbors=5, metric='cosine', algorithm='brute', device='cuda',
                 group=None):
        import torch.distributed as dist
        self._local = NearestNeighbors(n_neighbors, metric, algorithm, device)
        self.n_neighbors = n_neighbors
        self.device = self._local.device
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.lo = self.hi = 0
        self.n_samples_fit_ = None

    def fit(self, X, y=None):
        """X: the whole table (every rank passes the same one; only the
        rank's rows are copied to the device)."""
        n = X.shape[0]
        if n < self.world:
            raise ValueError(f"{n} rows cannot be split over {self.world} ranks")
        self.lo, self.hi = index_shard(n, self.rank, self.world)
        self._local.fit(X[self.lo:self.hi])
        self.n_samples_fit_ = n
        self.n_features_in_ = X.shape[1]
        return self

    def kneighbors_device(self, q: torch.Tensor, k: int):
        import torch.distributed as dist
        if self.n_samples_fit_ is None:
            raise RuntimeError("This ShardedNearestNeighbors instance is not fitted yet")
        if k > self.n_samples_fit_:
            raise ValueError(f"Expected n_neighbors <= n_samples_fit, but n_neighbors = {k}, "
                             f"n_samples_fit = {self.n_samples_fit_}")
        q = q.to(self.device, torch.float32).reshape(-1, self.n_features_in_).contiguous()
        Q = q.shape[0]
        kl = min(k, self.hi - self.lo)
        d_loc, i_loc = self._local.kneighbors_device(q, kl)
        dl = torch.full((Q, k), torch.finfo(torch.float32).max, dtype=torch.float32,
                        device=self.device)
        il = torch.full((Q, k), -1, dtype=torch.int64, device=self.device)
        dl[:, :kl] = d_loc
        il[:, :kl] = i_loc + self.lo
        dg = [torch.empty_like(dl) for _ in range(self.world)]
        ig = [torch.empty_like(il) for _ in range(self.world)]
        dist.all_gather(dg, dl, group=self.group)
        dist.all_gather(ig, il, group=self.group)
        dall = torch.stack(dg).contiguous()
        iall = torch.stack(ig).contiguous()
        idx = torch.empty((Q, k), dtype=torch.int64, device=self.device)
        dd = torch.empty((Q, k), dtype=torch.float32, device=self.device)
        lib = _lib.load()
        _lib.check(lib.dcnr_topk_merge(dall.data_ptr(), iall.data_ptr(), self.world, Q, k,
                                       idx.data_ptr(), dd.data_ptr(),
                                       _lib.stream_ptr(self.device)), "dcnr_topk_merge")
        return dd, idx

    def kneighbors(self, X=None, n_neighbors=None, return_distance=True):
        k = self.n_neighbors if n_neighbors is None else int(n_neighbors)
        if k <= 0:
            raise ValueError(f"Expected n_neighbors > 0. Got {k}")
        q = torch.as_tensor(np.asarray(X, dtype=np.float32)) if not torch.is_tensor(X) else X
        if q.shape[0] == 0:   # sklearn's check_array
            raise ValueError(f"Found array with 0 sample(s) (shape={tuple(q.shape)}) while a minimum "
                             "of 1 is required by NearestNeighbors.")
        dist_, idx = self.kneighbors_device(q, k)
        idx_np = idx.cpu().numpy()
        if return_distance:
            return dist_.cpu().numpy(), idx_np
        return idx_np
