"""Data-parallel path on CPU: world_size-2 gloo process groups (the GPU box runs
the same code over RCCL).  Covers the batch split, the flat-gradient exchange
convention (BCE grad pre-scaled by 1/world, SUM all-reduce == global mean) and
the SyncBN hook (pointer -> workspace view -> all-reduce) including the
statistics protocol libdcnr hands it (shifted sums unshifted, + count)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dcnr_oracle as orc
from dcnr import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _run(fn, world=2, *extra):
    port = _free_port()
    mp.spawn(fn, args=(world, port) + tuple(extra), nprocs=world, join=True)


def test_shard_range():
    assert parallel.shard_range(10, 0, 2) == (0, 5)
    assert parallel.shard_range(10, 1, 2) == (5, 10)
    assert parallel.shard_range(11, 1, 2) == (5, 10)   # ragged tail dropped
    lo_hi = [parallel.shard_range(131072 * 8, r, 8) for r in range(8)]
    assert lo_hi[0][0] == 0 and lo_hi[-1][1] == 131072 * 8
    assert all(a[1] == b[0] for a, b in zip(lo_hi, lo_hi[1:]))
    with pytest.raises(ValueError):
        parallel.shard_range(4, 2, 2)


def test_index_shard_covers_every_row():
    from dcnr.knn import index_shard
    for n, w in [(15, 2), (1_000_000, 8), (8, 8), (1_000_003, 7)]:
        parts = [index_shard(n, r, w) for r in range(w)]
        assert parts[0][0] == 0 and parts[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1
    with pytest.raises(ValueError):
        index_shard(4, 2, 2)


class _FakeModel:
    _active_ws = None
    bn_allreduce = None


def _hook_worker(rank, world, port):
    _init(rank, world, port)
    try:
        model = _FakeModel()
        hook = parallel.install_sync_bn(model)
        ws = torch.zeros(4096, dtype=torch.uint8)
        H = 24
        off = 512  # 256-aligned like libdcnr's bump allocator
        buf = ws[off:off + (3 * H + 1) * 8].view(torch.float64)
        rng = np.random.default_rng(rank)
        vals = rng.standard_normal(3 * H + 1)
        buf.copy_(torch.from_numpy(vals))
        model._active_ws = ws
        # through the ctypes thunk exactly as libdcnr calls it
        rc = hook.cfunc(None, ws.data_ptr() + off, 3 * H + 1, None)
        assert rc == 0 and hook.error is None and hook.calls == 1
        want = sum(np.random.default_rng(r).standard_normal(3 * H + 1) for r in range(world))
        np.testing.assert_allclose(buf.numpy(), want, rtol=0, atol=1e-12)
        # a pointer outside the active workspace is reported, not crashed on
        rc = hook.cfunc(None, ws.data_ptr() + 8192, 4, None)
        assert rc == 1 and isinstance(hook.error, RuntimeError)
        model._active_ws = None
        parallel.remove_sync_bn(model)
        assert model.bn_allreduce is None
    finally:
        dist.destroy_process_group()


def test_sync_bn_hook_gloo_world2():
    _run(_hook_worker)


def _stats_worker(rank, world, port):
    """SyncBN protocol: each rank produces [S0, S1, -, count] from ITS shard the
    way libdcnr does (sums shifted by the shard's first row, unshifted in fp64);
    after the hook's SUM the finalize (mean = S0/n, var = S1/n - mean^2) must
    equal BatchNorm statistics of the concatenated global batch."""
    _init(rank, world, port)
    try:
        B, H = 64, 16
        rng = np.random.default_rng(7)
        t_all = (rng.standard_normal((B * world, H)) * 0.3 + 50.0).astype(np.float32)
        lo, hi = parallel.shard_range(B * world, rank, world)
        t = t_all[lo:hi]
        K = t[0].astype(np.float64)
        d = t.astype(np.float64) - K
        s0p, s1p = d.sum(0), (d * d).sum(0)
        n = float(hi - lo)
        s1 = s1p + 2 * K * s0p + n * K * K
        s0 = s0p + n * K
        buf = torch.from_numpy(np.concatenate([s0, s1, np.zeros(H), [n]]))
        dist.all_reduce(buf)
        v = buf.numpy()
        cnt = v[3 * H]
        mean = v[:H] / cnt
        var = v[H:2 * H] / cnt - mean * mean
        np.testing.assert_allclose(cnt, B * world)
        np.testing.assert_allclose(mean, t_all.astype(np.float64).mean(0), rtol=1e-12)
        np.testing.assert_allclose(var, t_all.astype(np.float64).var(0), rtol=1e-6)
    finally:
        dist.destroy_process_group()


def test_sync_bn_statistics_protocol_gloo_world2():
    _run(_stats_worker)


def _random_params(spec, rng):
    """Random fp32 parameters keyed like the reference state_dict (train.py:136-153)."""
    D = orc.input_dim(spec.emb_dim, spec.cat_dims, spec.n_num)
    H = spec.hidden
    r = lambda *s: (rng.standard_normal(s) * 0.3).astype(np.float32)
    p = {"user_embedding.weight": r(spec.n_users, spec.emb_dim),
         "item_embedding.weight": r(spec.n_items, spec.emb_dim)}
    for k, n in enumerate(spec.cat_dims):
        p[f"cat_embeddings.{k}.weight"] = r(n, orc.cat_width(n))
    p["initial_deep_layer.weight"], p["initial_deep_layer.bias"] = r(H, D), r(H)
    for j in range(spec.n_res):
        for l in (1, 2):
            pre = f"res_blocks.{j}"
            p[f"{pre}.layer{l}.weight"], p[f"{pre}.layer{l}.bias"] = r(H, H), r(H)
            p[f"{pre}.bn{l}.weight"], p[f"{pre}.bn{l}.bias"] = 1 + r(H), r(H)
            p[f"{pre}.bn{l}.running_mean"] = r(H)
            p[f"{pre}.bn{l}.running_var"] = (1 + np.abs(r(H))).astype(np.float32)
            p[f"{pre}.bn{l}.num_batches_tracked"] = np.array(0)
    for l in range(spec.n_cross):
        p[f"cross_network.{l}.b"], p[f"cross_network.{l}.w.weight"] = r(D), r(1, D)
    p["final_linear.weight"], p["final_linear.bias"] = r(1, H + D), r(1)
    return p


def _grad_worker(rank, world, port):
    """Gradient exchange convention of FusedTrainer.step on the oracle model:
    every rank backpropagates (1/world) * mean-BCE of its shard; the SUM
    all-reduce of the flat gradient must equal the mean of the per-rank
    gradients, and with BN in eval mode (no batch coupling) the gradient of
    the global-batch loss."""
    _init(rank, world, port)
    try:
        spec = orc.ModelSpec(n_users=50, n_items=40, cat_dims=[7, 30], n_num=3, emb_dim=4,
                             hidden=16, n_cross=2, n_res=1, dropout=0.0)
        params = _random_params(spec, np.random.default_rng(3))
        rng = np.random.default_rng(11)
        Bg = 32
        user = rng.integers(0, 50, Bg); item = rng.integers(0, 40, Bg)
        cat = np.stack([rng.integers(0, 7, Bg), rng.integers(0, 30, Bg)], 1)
        num = rng.random((Bg, 3)); y = (rng.random(Bg) < 0.4).astype(np.float64)
        lo, hi = parallel.shard_range(Bg, rank, world)

        def grads(sl, scale):
            z, cache = orc.forward(params, spec, user[sl], item[sl], cat[sl], num[sl], train=False)
            _, dz = orc.bce_with_logits(z, y[sl])
            g = orc.backward(params, spec, cache, dz * scale, user[sl], item[sl], cat[sl])
            return np.concatenate([g[k].reshape(-1) for k in sorted(g)])

        local = torch.from_numpy(grads(slice(lo, hi), 1.0 / world))
        dist.all_reduce(local)
        full = grads(slice(0, Bg), 1.0)
        np.testing.assert_allclose(local.numpy(), full, rtol=1e-9, atol=1e-12)
    finally:
        dist.destroy_process_group()


def test_dp_gradient_exchange_gloo_world2():
    _run(_grad_worker)


def _host_adam(p, g, m, v, step, lr=1e-2, b1=0.9, b2=0.999, eps=1e-8, wd=1e-2):
    """torch.optim.AdamW's update (train.py:201-204) on host tensors, in place."""
    p.mul_(1 - lr * wd)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    denom = (v.sqrt() / (1 - b2 ** step) ** 0.5).add_(eps)
    p.addcdiv_(m, denom, value=-lr / (1 - b1 ** step))


def _exchange_worker(rank, world, port):
    _init(rank, world, port)
    try:
        import dcnr
        finals = {}
        for shard, chunks in ((True, 4), (True, 1), (True, 3), (False, 4)):
            torch.manual_seed(0)
            m = dcnr.DCN_RecSys(50, 40, {"a": 10, "b": 3}, 3,
                                dict(emb_dim=8, hidden_dim=16, n_cross_layers=1, n_res_blocks=1,
                                     dropout=0.0))
            tr = dcnr.FusedTrainer(m, lr=1e-2, weight_decay=1e-2, shard_optimizer=shard,
                                   exchange_chunks=chunks)
            assert tr.flat.numel() % (64 * world) == 0 and tr.E % (64 * world) == 0
            assert tr.chunks == (chunks if shard else 1)
            # the owned pieces: one per chunk, together 1/world of the segment
            rng = tr.shard_ranges()
            assert len(rng) == (chunks if shard else 0)
            assert sum(hi - lo for lo, hi in rng) == (tr.E // world if shard else 0)
            # the embedding segment's moments are sharded, the dense segment's whole
            assert tr.m.numel() == tr.E // (world if shard else 1) + tr.flat.numel() - tr.E
            ref_p = tr.flat.clone()
            ref_m = torch.zeros_like(ref_p)
            ref_v = torch.zeros_like(ref_p)
            for step in range(1, 4):
                # per parameter (not per flat position: the padding depends on
                # the chunk count), zeros in the padding
                grads = []
                for r in range(world):
                    gg = torch.zeros(tr.flat.numel())
                    for k, p in enumerate(m.param_tensors()):
                        o = (p.data_ptr() - tr.flat.data_ptr()) // 4
                        gen = torch.Generator().manual_seed(1000 * step + 10 * k + r)
                        gg[o:o + p.numel()] = torch.randn(p.numel(), generator=gen)
                    grads.append(gg)
                tr.gflat.copy_(grads[rank])
                tr.exchange_and_update(adam=_host_adam)
                _host_adam(ref_p, sum(grads), ref_m, ref_v, step)
                np.testing.assert_allclose(tr.flat.numpy(), ref_p.numpy(), rtol=2e-6, atol=1e-7)
                # every rank holds the same parameters, bit for bit
                allp = [torch.empty_like(tr.flat) for _ in range(world)]
                dist.all_gather(allp, tr.flat)
                assert all(torch.equal(allp[0], a) for a in allp[1:])
            # the module's parameters are views of the exchanged flat buffer
            assert m.final_linear.weight.data_ptr() >= tr.flat.data_ptr()
            finals[(shard, chunks)] = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        if world == 2:   # a sum of two is order-free: chunking changes no bit
            assert torch.equal(finals[(True, 4)], finals[(True, 1)])
            assert torch.equal(finals[(True, 3)], finals[(True, 1)])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_optimizer_exchange_matches_allreduce_adam(world):
    """FusedTrainer's data-parallel exchange (reduce-scatter -> AdamW on the
    rank's shard -> all-gather, and the all-reduce variant) gives every rank
    the single-process AdamW update of the summed gradient."""
    _run(_exchange_worker, world)


class HostSparseOps:
    """Host restatement of libdcnr's sparse-exchange kernels (dcnr_sparse_pack:
    the tables' touched rows in flat order; dcnr_sparse_accumulate: zero,
    then every source's rows added in rank order) -- the CPU side of the
    protocol test; the GPU tests run the kernels."""

    def pack(self, grad, offsets, table_counts, width, n_rows):
        tc = table_counts.tolist()
        off = torch.cat([offsets[t, :tc[t]] for t in range(len(tc))])
        assert off.numel() == n_rows
        col = torch.arange(width, dtype=torch.int64)
        rows = grad[off[:, None] + col[None, :]] if n_rows else torch.empty((0, width))
        return off, rows

    def accumulate(self, shard, lo, width, offsets, rows, counts):
        shard.zero_()
        sv = shard.view(-1, width)
        pos = 0
        for c in counts:
            if c:
                sv.index_add_(0, torch.div(offsets[pos:pos + c] - lo, width, rounding_mode="floor"),
                              rows[pos:pos + c])
            pos += c


def _sparse_worker(rank, world, port, d):
    """Owner-bucketed sparse exchange of the user and item tables
    (FusedTrainer exchange="sparse"): each rank's table gradients are nonzero
    only on its batch's ids (what dcnr_backward writes); after the exchange
    the owner's shard holds the dense SUM, bit for bit (summed in rank
    order), and the AdamW step matches the single-process update."""
    _init(rank, world, port)
    try:
        import dcnr
        n_users = 257
        ids = [torch.randint(0, n_users, (40,), generator=torch.Generator().manual_seed(50 + r))
               for r in range(world)]
        ids[world - 1][:5] = n_users - 1          # the last owner's tail row
        # through FusedTrainer(exchange="sparse"): the user and item tables'
        # touched rows go to the owners of their ZeRO-1 shard
        # (sparse_reduce_scatter), the categorical tables through an
        # all-reduce; AdamW on the shard, all-gather of the parameters
        n_items = 40
        torch.manual_seed(0)
        m = dcnr.DCN_RecSys(n_users, n_items, {"a": 10, "b": 3}, 3,
                            dict(emb_dim=d, hidden_dim=16, n_cross_layers=1, n_res_blocks=1,
                                 dropout=0.0))
        tr = dcnr.FusedTrainer(m, lr=1e-2, weight_decay=1e-2, exchange="sparse",
                               sparse_ops=HostSparseOps())
        assert tr.shard and tr.m.numel() == tr.E // world + tr.flat.numel() - tr.E
        lay = tr._sparse_layout
        nu = lay["elem_off"][1]
        iids = [torch.randint(0, n_items, (40,), generator=torch.Generator().manual_seed(80 + r))
                for r in range(world)]
        ref_p, ref_m, ref_v = tr.flat.clone(), torch.zeros_like(tr.flat), torch.zeros_like(tr.flat)
        for step in range(1, 3):
            full, touched = [], []
            for r in range(world):
                gg = torch.randn(tr.flat.numel(), generator=torch.Generator().manual_seed(9 * step + r))
                gg[:lay["dense_lo"]] = 0          # the sparse tables: touched rows only
                offs = torch.zeros((2, 40), dtype=torch.int64)
                tcnt = torch.zeros(2, dtype=torch.int64)
                for t, (ids_t, base) in enumerate(((ids[r], 0), (iids[r], nu))):
                    u = torch.unique(ids_t) * d + base     # what dcnr_emb_touched_rows returns
                    for o in u.tolist():
                        gg[o:o + d] = torch.randn(d, generator=torch.Generator().manual_seed(o + r))
                    offs[t, :u.numel()] = u
                    tcnt[t] = u.numel()
                own = torch.bincount(torch.cat([offs[t, :tcnt[t]] for t in range(2)]) // tr.Es,
                                     minlength=world)
                full.append(gg)
                touched.append((offs, tcnt, own))
            tr.gflat.copy_(full[rank])
            tr.exchange_and_update(adam=_host_adam, touched=touched[rank])
            want = sum(full)
            lo, hi = rank * tr.Es, (rank + 1) * tr.Es
            sp = min(hi, lay["dense_lo"])
            if sp > lo:   # the sparse tables' part of the shard: the rank-order sum, bit for bit
                assert torch.equal(tr.gshard[:sp - lo], want[lo:sp])
            np.testing.assert_allclose(tr.gshard.numpy(), want[lo:hi].numpy(), rtol=1e-6, atol=1e-7)
            _host_adam(ref_p, want, ref_m, ref_v, step)
            np.testing.assert_allclose(tr.flat.numpy(), ref_p.numpy(), rtol=2e-6, atol=1e-7)
            allp = [torch.empty_like(tr.flat) for _ in range(world)]
            dist.all_gather(allp, tr.flat)
            assert all(torch.equal(allp[0], a) for a in allp[1:])
            assert tr.last_exchange["rows_sent"] == int(sum(c for c in touched[rank][1]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,d", [(2, 8), (3, 8), (2, 24), (3, 48)])
def test_sparse_user_table_exchange(world, d):
    """emb_dim 24 / 48 (in the reference's Optuna space, train.py:180): the
    tables and the shards are padded to lcm(64, emb_dim) so rows never
    straddle a shard."""
    _run(_sparse_worker, world, d)


def test_sparse_exchange_argument_checks():
    import dcnr
    m = dcnr.DCN_RecSys(50, 40, {"a": 10}, 3, dict(emb_dim=8, hidden_dim=16, n_cross_layers=1,
                                                     n_res_blocks=1, dropout=0.0))
    with pytest.raises(ValueError):
        dcnr.FusedTrainer(m, exchange="sparse", shard_optimizer=False)
