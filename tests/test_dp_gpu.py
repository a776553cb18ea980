"""Data-parallel step on the device (a world-2 DP step with
SyncBN equals the single-process step at the global batch).

Two ranks share cuda:0 over gloo (RCCL refuses two ranks on one device; the
exchange code is backend-agnostic: FusedTrainer pre-scales the BCE gradient
by 1/world and SUM-reduces the flat gradient, SyncBN sums each BatchNorm's
fp64 statistics buffer across ranks inside the native forward/backward).
Rank r trains on rows [r*B/2, (r+1)*B/2) of the batch the single process
trains on whole.  After one step the summed gradient, the logits, the BN
running statistics and the updated parameters must match the single-process
step (dropout 0: the counter-based dropout mask is a function of the local
row index), in fp32 (tight bounds) and in bf16 -- the benchmarked N>1 path,
where the backward's weight gradients run on the library's side stream and
are joined before the DCNR_GRADS_DENSE hook starts the all-reduce (bounds of
test_bf16_train_gpu: cos >= 0.98, rel <= 0.25 per tensor; running stats
1e-2).

test_dp_bf16_hook_ordering pins that join at dropout 0.6: the dense segment
each rank holds after the exchange the hook started must be bit-identical to
an explicit all-reduce of the same ranks' gradients from a second, identical
step run without the hook (the side stream then joins at the end of the
backward); likewise the embedding segment (all-reduce or reduce-scatter).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import golden_common as gc

pytestmark = pytest.mark.gpu

CFG = dict(n_users=3000, n_items=700, cat_dims={"a": 50, "b": 1000, "c": 7}, n_num=5,
           params=dict(emb_dim=16, hidden_dim=128, n_cross_layers=2, n_res_blocks=2,
                       dropout=0.0))
B = 2048
# BASELINE configs[3] per rank: the bench model (1M x 32 users, 100k x 32
# items, 12 x 1000 x 32 categorical, 8 dense, 3 cross, 4 x 512 deep) at the
# bench's 131072 samples per rank -- two ranks on one GPU (3.8 GB of
# workspace each), so the global batch is 262144
BENCH = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{i}": 1000 for i in range(12)}, n_num=8,
             params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4, dropout=0.0))
CONFIGS = {"toy": (CFG, B), "bench": (BENCH, 2 * 131072)}


def _model(dev, precision="fp32", dropout=0.0, cfg=CFG):
    import dcnr
    torch.manual_seed(5)
    params = dict(cfg["params"], dropout=dropout)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        params, precision=precision)
    gc.perturb_state(m, 6)
    return m.to(dev)


def _cos_rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    cos = (a @ b / (a.norm() * b.norm()).clamp_min(1e-300)).item()
    rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
    return cos, rel


def _batch(dev, cfg=CFG, nb=B, seed=123):
    u, i, c, n, y = gc.make_inputs(cfg, nb, seed)
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (u, i, c, n, y)]


def _worker(rank, world, port, path, shard, precision):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcnr
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        m = _model(dev, precision)
        tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4, sync_bn=True,
                               shard_optimizer=shard)
        seen = []
        hook = tr._on_grads_ready

        def spy(ctx, group, stream):   # the backward's gradient-group hook fired, in order
            seen.append(group)
            return hook(ctx, group, stream)
        tr._on_grads_ready = spy
        tr._grad_ready_cb = dcnr._lib.GRAD_READY_FN(spy)
        lo, hi = rank * B // world, (rank + 1) * B // world
        batch = [t[lo:hi] for t in _batch(dev)]
        loss, z = tr.step(*batch, return_logits=True)
        torch.cuda.synchronize()
        assert seen == [dcnr._lib.GRADS_DENSE, dcnr._lib.GRADS_EMBEDDING], seen
        zs = [torch.empty_like(z) for _ in range(world)]
        dist.all_gather(zs, z.contiguous())
        if rank == 0 and precision == "bf16":
            ref = torch.load(path, weights_only=True)
            zz = torch.cat(zs).cpu().double()
            assert (zz - ref["z"]).abs().max().item() <= 2e-2 * max(1.0, ref["z"].abs().max().item())
            bad = []
            for k, p in m.named_parameters():   # the exchanged (summed) gradients
                if ".layer" in k and k.endswith(".bias"):    # BN-invariant: ~0
                    continue
                if shard and "embedding" in k:   # reduce-scattered into tr.gshard
                    continue
                cos, rel = _cos_rel(p.grad.cpu(), ref["grads"][k])
                if cos < 0.98 or rel > 0.25:
                    bad.append((k, cos, rel))
            assert not bad, bad
            for k, v in m.state_dict().items():
                if "running" in k:
                    np.testing.assert_allclose(v.cpu().numpy(), ref["sd"][k].numpy(),
                                               rtol=1e-2, atol=1e-2, err_msg=k)
                if "num_batches_tracked" in k:
                    assert int(v) == int(ref["sd"][k]) == 1
        elif rank == 0:
            ref = torch.load(path, weights_only=True)
            zz = torch.cat(zs).cpu().double()
            assert (zz - ref["z"]).abs().max().item() <= 1e-5 * max(1.0, ref["z"].abs().max().item())
            names = [k for k, _ in m.named_parameters()]
            bad = []
            for k, p in m.named_parameters():   # the exchanged (summed) gradients
                a, b = p.grad.cpu().double().reshape(-1), ref["grads"][k].reshape(-1)
                if ".layer" in k and k.endswith(".bias"):    # BN-invariant: ~0
                    continue
                if shard and "embedding" in k:   # reduce-scattered into tr.gshard, not
                    continue                     # into p.grad: the params check covers it
                e = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
                if e > 1e-4:
                    bad.append((k, e))
            assert not bad, bad
            for k, v in m.state_dict().items():
                if k in ref["params"] and not (".layer" in k and k.endswith(".bias")):
                    # the AdamW step on the exchanged gradient: its first update is
                    # ~lr * sign(g), so an element whose summed gradient is pure
                    # rounding noise may move the other way -- allow 0.1 % of them
                    d = (v.cpu().double() - ref["params"][k].double()).abs()
                    frac = (d > 1e-6).double().mean().item()
                    assert frac <= 1e-3 and d.max().item() <= 2.5e-3, (k, frac)
                if "running" in k:
                    np.testing.assert_allclose(v.cpu().numpy(), ref["sd"][k].numpy(),
                                               rtol=1e-5, atol=1e-6, err_msg=k)
                if "num_batches_tracked" in k:
                    assert int(v) == int(ref["sd"][k]) == 1
            assert len(names) > 0
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("shard", [False, True])
def test_dp_world2_syncbn_equals_single_process(dev, shard, precision):
    """shard=True: the embedding segment goes through reduce-scatter -> shard
    AdamW -> all-gather, the dense segment's all-reduce is started by the
    backward's DCNR_GRADS_DENSE hook; shard=False: all-reduce of both."""
    import dcnr
    m = _model(dev, precision)
    tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4)
    batch = _batch(dev)
    loss, z = tr.step(*batch, return_logits=True)
    torch.cuda.synchronize()
    ref = {"z": z.detach().cpu().double(),
           "grads": {k: p.grad.detach().cpu().double().clone() for k, p in m.named_parameters()},
           "params": {k: p.detach().cpu().clone() for k, p in m.named_parameters()},
           "sd": {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}}
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ref.pt")
        torch.save(ref, path)
        mp.spawn(_worker, args=(2, _free_port(), path, shard, precision), nprocs=2, join=True)


def _worker_hook(rank, world, port, shard, cfg_name="toy", sync_bn=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcnr
        from dcnr.model import dropout_seed, run_backward, run_forward
        from dcnr.ops import bce_with_logits
        cfg, nb = CONFIGS[cfg_name]
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        m = _model(dev, "bf16", dropout=0.6, cfg=cfg)
        tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4, sync_bn=sync_bn,
                               shard_optimizer=shard)
        lo, hi = rank * nb // world, (rank + 1) * nb // world
        u, i, c, n, y = [t[lo:hi] for t in _batch(dev, cfg, nb)]
        gen = torch.cuda.default_generators[0]
        off0 = gen.get_offset()
        flat0 = tr.flat.clone()
        bufs0 = {k: v.clone() for k, v in m.named_buffers()}
        # 1) the trainer's step: the hook starts the dense all-reduce inside
        #    the backward, right after the side stream's weight gradients join
        tr.step(u, i, c, n, y)
        torch.cuda.synchronize()
        E = tr.E
        dense_hook = tr.gflat[E:].clone()
        emb_hook = (tr.gshard if shard else tr.gflat[:E]).clone()
        # 2) the same step (same parameters, running stats, dropout seed) with
        #    no hook: the backward joins its side stream at the end; then an
        #    explicit all-reduce of the local gradients
        tr.flat.copy_(flat0)
        for k, v in m.named_buffers():
            v.copy_(bufs0[k])
        gen.set_offset(off0)
        seed = dropout_seed(dev)
        uu, ii, cc, nn_ = m.prepare_inputs(u, i, c, n)
        logits, ws = run_forward(m, True, seed, uu, ii, cc, nn_)
        _, dz = bce_with_logits(logits, y.reshape(-1).float().contiguous(), True, 1.0 / world)
        run_backward(m, uu, ii, cc, nn_, dz, ws, tr._grads, seed, accumulate=False)
        torch.cuda.synchronize()
        g = tr.gflat.clone()
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        assert torch.equal(dense_hook, g[E:]), "dense segment: hook exchange != explicit all-reduce"
        Es = tr.Es
        emb_ref = torch.cat([g[lo:hi] for lo, hi in tr.shard_ranges()]) if shard else g[:E]
        assert not shard or sum(hi - lo for lo, hi in tr.shard_ranges()) == Es
        assert torch.equal(emb_hook, emb_ref), "embedding segment differs"
        assert dense_hook.abs().sum().item() > 0
        if cfg_name == "bench":   # the shard boundary of the 142 MB table segment
            assert E % (64 * world) == 0 and E >= sum(p.numel() for p in m.param_tensors()[:14])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shard", [False, True])
def test_dp_bf16_hook_ordering(dev, shard):
    """configs[3]'s path in one-GPU rehearsal form: bf16, dropout 0.6, SyncBN,
    side-stream weight gradients, the grad-ready hook, sharded or all-reduce
    exchange (train.py:219-226)."""
    mp.spawn(_worker_hook, args=(2, _free_port(), shard), nprocs=2, join=True)


@pytest.mark.parametrize("shard", [False, True])
def test_dp_bf16_hook_ordering_bench_model(dev, shard):
    """The same pin at BASELINE configs[3]'s per-rank workload: the bench
    model (1M-row user table, 4 x 512 deep, bf16, dropout 0.6) at 131072
    samples per rank, local BN as the bench runs it: the 142 MB embedding
    segment's shards, the side-stream weight-gradient pipe at 4 blocks of
    512 and the hook firing before the dx0 GEMM (train.py:219-226)."""
    mp.spawn(_worker_hook, args=(2, _free_port(), shard, "bench", False), nprocs=2, join=True)


def _worker_sparse(rank, world, port, cfg_name="toy", sync_bn=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dcnr
        cfg, nb = CONFIGS[cfg_name]
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        lo, hi = rank * nb // world, (rank + 1) * nb // world
        flats = []
        # "sparse" writes only the touched table rows in the backward (row
        # map, no zero fill); "sparse-zerofill" keeps the zero-filled tables
        runs = ("dense", "sparse") + (("sparse-zerofill",) if cfg_name == "toy" else ())
        for run in runs:
            exchange = run.split("-")[0]
            m = _model(dev, "bf16", dropout=0.6, cfg=cfg)
            tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4, sync_bn=sync_bn, exchange=exchange,
                                   dense_table_grads=run.endswith("zerofill"))
            assert tr._sparse_rows() == (run == "sparse")
            gen = torch.cuda.default_generators[0]
            gen.set_offset(0)                      # the same dropout seeds in both runs
            for step in range(2):
                batch = [t[lo:hi] for t in _batch(dev, cfg, nb, 123 + step)]
                tr.step(*batch)
                if exchange == "sparse" and step == 0:
                    # the touched rows of this rank's batch, from the backward's sort
                    offs, tcnt, own = tr.touched_rows()
                    lay = tr._sparse_layout
                    d = lay["width"]
                    want = [torch.unique(batch[0].long()) * d,
                            torch.unique(batch[1].long()) * d + lay["elem_off"][1]]
                    tc = tcnt.cpu().tolist()
                    for t in range(2):
                        assert torch.equal(offs[t, :tc[t]], want[t]), t
                    allw = torch.cat(want)
                    assert torch.equal(own.cpu(), torch.bincount((allw // tr.Es).cpu(),
                                                                 minlength=world))
            torch.cuda.synchronize()
            # per parameter: the dense exchange's chunked layout pads the
            # table segment differently from the sparse exchange's
            flats.append(torch.cat([p.detach().reshape(-1) for p in m.param_tensors()]))
            assert tr.exchange != "sparse" or tr.last_exchange["rows_sent"] > 0
            del tr, m
            torch.cuda.empty_cache()
        # world 2: the owner's rank-order sum (0 + g_0) + g_1 is the dense
        # reduce-scatter's g_0 + g_1: every parameter bit-identical
        for f in flats[1:]:
            assert torch.equal(flats[0], f)
    finally:
        dist.destroy_process_group()


def test_dp_sparse_exchange_equals_dense(dev):
    """exchange="sparse" (touched rows from the backward's sort ->
    all_to_all to the shard owners -> rank-order sums; categorical tables
    all-reduced) gives exactly the dense reduce-scatter step: bf16, dropout
    0.6, SyncBN, two steps, two ranks on one GPU (train.py:156-158, 225)."""
    mp.spawn(_worker_sparse, args=(2, _free_port()), nprocs=2, join=True)


def test_dp_sparse_exchange_equals_dense_bench_model(dev):
    """The sparse exchange at BASELINE configs[3]'s per-rank workload: the
    1M-row user and 100k-row item tables' touched rows (~123k + 73k per
    rank) equal torch.unique of the batch, and two steps give every
    parameter bit-identical to the dense reduce-scatter's (train.py:156-158,
    225)."""
    mp.spawn(_worker_sparse, args=(2, _free_port(), "bench", False), nprocs=2, join=True)
