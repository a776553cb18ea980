"""Row-sharded cosine index (each rank scans N/world
rows, all-gather of the world*k candidates, one merge): bit-identical to the
single index over the whole table, ties included.

The merge kernel (``dcnr_topk_merge``) is checked against a numpy lexsort on
lists with planted distance ties and padding; the sharded index runs as two
processes sharing cuda:0 over gloo (RCCL refuses two ranks on one device; the
exchange is backend-agnostic) and must return exactly the single-process
``NearestNeighbors`` result -- the scan2 path (Q < 32) and the MFMA scan3 path
(Q >= 32), duplicate rows split across the two shards, and a table whose
shards hold fewer than k rows each.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _merge_ref(d, i, k):
    """numpy: the k best of [L][Q][k] by (dist, row as uint64)."""
    L, Q, _ = d.shape
    dd = np.transpose(d, (1, 0, 2)).reshape(Q, -1)
    ii = np.transpose(i, (1, 0, 2)).reshape(Q, -1).astype(np.uint64)
    od, oi = np.empty((Q, k), np.float32), np.empty((Q, k), np.int64)
    for q in range(Q):
        o = np.lexsort((ii[q], dd[q]))[:k]
        od[q], oi[q] = dd[q][o], ii[q][o].astype(np.int64)
    return od, oi


@pytest.mark.parametrize("L,k", [(2, 11), (8, 11), (3, 64), (32, 64)])
def test_topk_merge_matches_lexsort(dev, L, k):
    from dcnr import _lib
    rng = np.random.default_rng(L * 100 + k)
    Q = 37
    d = rng.integers(0, 50, (L, Q, k)).astype(np.float32) / 64   # many exact ties
    i = rng.permutation(L * Q * k * 4)[:L * Q * k].reshape(L, Q, k).astype(np.int64)
    d[0, :, -1] = np.finfo(np.float32).max   # padding entries
    i[0, :, -1] = -1
    od, oi = _merge_ref(d, i, k)
    dt, it = torch.from_numpy(d).to(dev), torch.from_numpy(i).to(dev)
    gi = torch.empty((Q, k), dtype=torch.int64, device=dev)
    gd = torch.empty((Q, k), dtype=torch.float32, device=dev)
    lib = _lib.load()
    _lib.check(lib.dcnr_topk_merge(dt.data_ptr(), it.data_ptr(), L, Q, k, gi.data_ptr(),
                                   gd.data_ptr(), _lib.stream_ptr(dev)), "merge")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gd.cpu().numpy(), od)
    np.testing.assert_array_equal(gi.cpu().numpy(), oi)


def test_topk_merge_rejects_oversize(dev):
    from dcnr import _lib
    lib = _lib.load()
    t = torch.zeros(16, device=dev)
    st = lib.dcnr_topk_merge(t.data_ptr(), t.data_ptr(), 64, 1, 64, t.data_ptr(), t.data_ptr(),
                             _lib.stream_ptr(dev))
    assert st == _lib.DCNR_UNSUPPORTED_SHAPE


def _table(n, d, seed):
    rng = np.random.default_rng(seed)
    t = rng.standard_normal((n, d)).astype(np.float32)
    if n > 100:   # duplicates straddling the shard boundary: exact distance ties
        h = n // 2
        t[h - 3:h + 3] = t[7]
        t[n - 5:] = 2.5 * t[11]   # scaled copies: the same cosine
    return t


def _cases():
    # (60000 and 70001 rows: the whole table above scan v4's 32768-row sample,
    # each shard below it -- the same arithmetic either way)
    # (60000 / 70001 rows: the table above scan v4's 32768-row sample, each
    # shard below it; 1M rows at Q=1: the single index takes v4, its
    # 500000-row shards scan v2 -- the same distances either way)
    return [(20000, 64, 1), (20000, 64, 7), (20000, 64, 40), (5003, 32, 33), (15, 16, 3),
            (60000, 64, 40), (70001, 32, 1), (1_000_000, 64, 1)]


def _worker(rank, world, port, path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcnr
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        ref = torch.load(path, weights_only=True)
        for c, (n, d, Q) in enumerate(_cases()):
            tab = _table(n, d, c)
            nn = dcnr.ShardedNearestNeighbors(n_neighbors=11, device=dev).fit(tab)
            assert nn.hi - nn.lo in (n // world, n // world + 1)
            rng = np.random.default_rng(100 + c)
            q = tab[rng.integers(0, n, Q)] + 0.01 * rng.standard_normal((Q, d)).astype(np.float32)
            q[0] = tab[7]   # a query tied with the duplicates
            dd, ii = nn.kneighbors(q)
            np.testing.assert_array_equal(ii, ref[f"i{c}"].numpy(), err_msg=str((rank, c)))
            np.testing.assert_array_equal(dd, ref[f"d{c}"].numpy(), err_msg=str((rank, c)))
    finally:
        dist.destroy_process_group()


def test_sharded_index_equals_single_index(dev):
    import dcnr
    ref = {}
    for c, (n, d, Q) in enumerate(_cases()):
        tab = _table(n, d, c)
        nn = dcnr.NearestNeighbors(n_neighbors=11, device=dev).fit(tab)
        rng = np.random.default_rng(100 + c)
        q = tab[rng.integers(0, n, Q)] + 0.01 * rng.standard_normal((Q, d)).astype(np.float32)
        q[0] = tab[7]
        dd, ii = nn.kneighbors(q)
        ref[f"d{c}"], ref[f"i{c}"] = torch.from_numpy(dd), torch.from_numpy(ii)
        if n > 100:   # the planted ties are in the answer
            assert len(set(ii[0].tolist()) & set(range(n // 2 - 3, n // 2 + 3))) > 0
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ref.pt")
        torch.save(ref, path)
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        mp.spawn(_worker, args=(2, port, path), nprocs=2, join=True)


def _bench_worker(rank, world, port):
    import sys
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        out = bench.bench_cfg5_sharded(dev, 1, world)
        assert all(out[f"topk_q{Q}_us"] > 0 for Q in (1, 32, 256)), out
    finally:
        dist.destroy_process_group()


def test_bench_sharded_leg_runs_world2():
    """bench.py's N > 1 sharded-index leg end to end (two ranks on cuda:0)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_bench_worker, args=(2, port), nprocs=2, join=True)
