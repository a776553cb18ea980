#!/usr/bin/env python
"""bench.py -- DCN-R training step on MI355X (BASELINE.json configs[2] / [3]).

One step = one pass of the hot path over one synthetic batch per GPU:
    forward (train-mode BN, dropout 0.6) -> BCEWithLogits -> backward
    -> [RCCL all-reduce of the flat gradient when N > 1] -> fused AdamW
Workload (BASELINE.json configs[2]): 1M users x 100k hotels, 12 categorical
tables of 1000 rows (width 32), 8 dense features, emb_dim 32, 3 cross layers,
4 x 512 residual deep tower, batch 131072 per GPU, bf16 MFMA deep tower with
fp32 accumulation / fp32 master weights.  N > 1 is configs[3] (data parallel,
weak scaling: per-GPU batch fixed).  Inputs are pre-generated on the device
(fresh ids every step from a pool), weights seed 42, inputs seed 0 (+rank).

Run: python bench.py [--gpus N --steps K --warmup W]; N > 1 under
torch.distributed.run (one process per GPU, RCCL).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CFG = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
           n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4,
                                dropout=0.6))
D, H, R = 456, 512, 4
GEMM_FLOP = {  # algorithmic FLOPs per sample per step (13.98 MFLOP fwd+bwd)
    "gemm_fwd": 2 * (D * H + 2 * R * H * H),
    "gemm_dx": 2 * (2 * R * H * H + H * D),
    "gemm_dw": 2 * (2 * R * H * H + H * D),
}
# eval forward (scoring) FLOPs per (user, hotel) pair: the deep tower's GEMMs
EVAL_FLOP_PER_PAIR = 2 * (D * H + 2 * R * H * H)
# gather + x0 + 3 cross: 14 idx x 8 B + 14 rows x 128 B + 8 x 4 B read; x0 bf16 + zc written
GATHER_BYTES = 14 * 8 + 14 * 32 * 4 + 8 * 4 + D * 2 + 4
# algorithmic HBM bytes of the forward Linear class per step: X read + C write
# (bf16) per sample, 9 launches (initial D -> H, then 2 x R H -> H), plus the
# bf16 weights once per launch
GEMM_FWD_BYTES_PER_SAMPLE = 2 * (D + H) + 2 * R * 2 * (H + H)
GEMM_FWD_W_BYTES = 2 * (H * D + 2 * R * H * H)
# BASELINE configs[1] (gather + x0 + 3 cross forward, fp32, B=65536): SURVEY 8d
# algorithmic bytes per sample = 14 ids x 8 B + 14 rows x 128 B + 8 x 4 B read
# (1936 B) + the fp32 cross_out row written (456 x 4 = 1824 B)
CFG2_B = 65536
CFG2_BYTES = 14 * 8 + 14 * 32 * 4 + 8 * 4 + D * 4
PEAK_BF16 = 2.5e15     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM = 8.0e12
SINGLE_KERNEL_CLASSES = ("gemm_dw", "adam", "gather_cross")
CLASS_KERNELS = {
    "gather_cross": "gather_cross_v4_kernel (train forward)",
    "gemm_fwd": "gemm_ws_kernel (deep-tower Linear forward)",
    "gemm_dx": "gemm_ws_kernel (deep-tower dX with BN-backward epilogues)",
    "gemm_dw": "gemm_dw_kernel (deep-tower weight gradient)",
    "rowwise": "rowcol_kernel (BN apply / statistics passes)",
    "reduce": "reduce / split-K combine kernels",
    "cross_bwd": "cross_coef / x0_alpha / cross_final kernels (low-rank cross backward)",
    "emb_sort": "emb_ids/hist/scan/scatter/bucket_sort kernels (stable id sort)",
    "emb_sum": "emb_runs_short/long_kernel (fixed-order embedding-gradient sums)",
    "head": "row_dot / head_parts / logits / bce kernels",
    "adam": "adam_kernel (fused AdamW)",
    "pack": "pack / zero-fill kernels",
    "tower": "tower_kernel (fused eval deep tower: 9 Linear + BN + ReLU + residual + head, one launch)",
}


def make_batch(gen, B, dev):
    ids = lambda n: torch.randint(0, n, (B,), generator=gen, device=dev, dtype=torch.int64)
    user = ids(CFG["n_users"])
    item = ids(CFG["n_items"])
    cat = torch.randint(0, 1000, (B, 12), generator=gen, device=dev, dtype=torch.int64)
    num = torch.rand((B, 8), generator=gen, device=dev, dtype=torch.float32)
    y = (torch.rand((B,), generator=gen, device=dev) < 0.5).float()
    return user, item, cat, num, y


class ZipfIds:
    """Ids with P(rank r) ~ r^-a over n rows (the secondary
    Zipf(1.05) distribution), ranks mapped to rows by a fixed permutation so
    the hot rows are scattered over the table."""

    def __init__(self, n, dev, a=1.05, seed=3):
        g = torch.Generator(device=dev).manual_seed(seed)
        w = torch.arange(1, n + 1, device=dev, dtype=torch.float64).pow(-a)
        self.cdf = torch.cumsum(w, 0) / w.sum()
        self.perm = torch.randperm(n, generator=g, device=dev)
        self.n = n

    def __call__(self, shape, gen, dev):
        u = torch.rand(shape, generator=gen, device=dev, dtype=torch.float64)
        r = torch.searchsorted(self.cdf, u).clamp_(max=self.n - 1)
        return self.perm[r]


def bench_zipf(trainer, dev, B, world, steps=10, warmup=3):
    """The train step on Zipf(1.05) ids for the user, item and categorical
    columns (fresh batch per step, generated before the timed region)."""
    gen = torch.Generator(device=dev).manual_seed(77 + (dist.get_rank() if world > 1 else 0))
    zu, zi, zc = ZipfIds(CFG["n_users"], dev), ZipfIds(CFG["n_items"], dev), ZipfIds(1000, dev)
    pool = []
    for _ in range(warmup + steps):
        pool.append((zu((B,), gen, dev), zi((B,), gen, dev), zc((B, 12), gen, dev),
                     torch.rand((B, 8), generator=gen, device=dev),
                     (torch.rand((B,), generator=gen, device=dev) < 0.5).float()))
    top_user = float(torch.bincount(pool[0][0]).max()) / B
    for k in range(warmup):
        trainer.step(*pool[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        trainer.step(*pool[warmup + k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    return {"distribution": "Zipf(1.05) over each table's rows (user, item, 12 categorical), "
                            "ranks scattered by a fixed permutation",
            "samples_per_sec": world * B * steps / el, "ms_per_step": el / steps * 1e3,
            "steps": steps, "top_user_share": top_user}


def cpu_threads():
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def cpu_baseline(B_cpu=32768, steps=3):
    """The reference's own training step (train.py:155-226: forward, BCE,
    backward, AdamW) as torch-CPU ops in the reference's order
    (oracle/torch_cpu.py, validated within 10 % of the imported reference by
    tools/validate_cpu_baseline.py), timed on the host cores at a bounded
    batch of the same model.  Reported only; not the optimisation target."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch_cpu as tc
    th = cpu_threads()
    torch.set_num_threads(th)
    cat = list(CFG["cat_dims"].values())
    p = CFG["params"]
    step = tc.TorchCPUStep(CFG["n_users"], CFG["n_items"], cat, CFG["n_num"], p["emb_dim"],
                           p["hidden_dim"], p["n_cross_layers"], p["n_res_blocks"], p["dropout"],
                           lr=1e-3, weight_decay=1e-4)
    batches = [tc.make_cpu_batch(CFG["n_users"], CFG["n_items"], cat, CFG["n_num"], B_cpu, k)
               for k in range(steps + 1)]
    t = tc.time_steps(step.step, batches, warmup=1)
    # scored pairs/s: the eval-mode forward (main.py:319-322) of the same model
    ts = tc.time_steps(lambda u, i, c, n, y: step.score(u, i, c, n), batches, warmup=1)
    del step, batches
    return {"value": B_cpu / t, "unit": "samples/s", "cores": th, "kind": "port",
            "scored_pairs": {"value": B_cpu / ts, "unit": "pairs/s", "cores": th, "kind": "port",
                             "sample": f"{steps} eval-mode forwards (running-stat BN, no dropout, "
                                       f"no_grad) at batch {B_cpu}, torch-CPU ops of "
                                       f"oracle/torch_cpu.py, {steps * ts:.1f} s"},
            "validated": "step time within 10 % of the imported reference train.py step on the "
                         "same host (tools/validate_cpu_baseline.py, profiles/r02_cpu_baseline.txt)",
            "sample": f"{steps} timed train steps (zero_grad, fwd, BCEWithLogits, bwd, AdamW) at "
                      f"batch {B_cpu} of the bench model, fp32 torch-CPU ops in train.py:155-226 "
                      f"order (oracle/torch_cpu.py), {steps * t:.1f} s",
            "numpy_port": cpu_port_baseline()}


def cpu_port_baseline(B_cpu=16384, steps=2):
    """Secondary figure: the numpy fp32 oracle (restatement of train.py:155-226)
    on the same model, forward + BCE + backward + AdamW."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dcnr_oracle as orc
    import dcnr
    torch.manual_seed(42)
    m = dcnr.DCN_RecSys(CFG["n_users"], CFG["n_items"], CFG["cat_dims"], CFG["n_num"],
                        dict(CFG["params"], dropout=0.0))
    sd = {k: v.detach().numpy().astype(np.float32) for k, v in m.state_dict().items()}
    del m
    spec = orc.spec_from_params(CFG["n_users"], CFG["n_items"], CFG["cat_dims"], CFG["n_num"],
                                dict(CFG["params"], dropout=0.0))
    rng = np.random.default_rng(0)
    names = [k for k in sd if "running" not in k and "num_batches" not in k]
    mom = {k: (np.zeros_like(sd[k]), np.zeros_like(sd[k])) for k in names}
    t0 = time.perf_counter()
    for s in range(steps):
        u = rng.integers(0, CFG["n_users"], B_cpu)
        i = rng.integers(0, CFG["n_items"], B_cpu)
        c = rng.integers(0, 1000, (B_cpu, 12))
        n = rng.random((B_cpu, 8), dtype=np.float32)
        y = (rng.random(B_cpu) < 0.5).astype(np.float32)
        z, cache = orc.forward(sd, spec, u, i, c, n, train=True, dt=np.float32)
        _, dz = orc.bce_with_logits(z, y)
        g = orc.backward(sd, spec, cache, dz.astype(np.float32), u, i, c, dt=np.float32)
        for k in names:
            p, mm, vv = orc.adam_step(sd[k], g[k], *mom[k], s + 1, 1e-3, weight_decay=1e-4)
            sd[k] = p.astype(np.float32)
            mom[k] = (mm, vv)
    el = time.perf_counter() - t0
    return {"value": steps * B_cpu / el, "unit": "samples/s", "kind": "port",
            "sample": f"{steps} steps at batch {B_cpu}, numpy fp32 oracle, {el:.1f} s"}


def bench_cfg2(model, gen, dev, iters, world):
    """BASELINE configs[1]: embedding gathers + x0 concat + 3 cross layers,
    fp32 cross_out [65536, 456], on the bench model's tables
    (DCN_RecSys.gather_cross -> dcnr_gather_cross).  Per-launch kernel time
    from HIP events on the launch stream (libdcnr profiling); wall time over
    `iters` back-to-back calls between synchronisations."""
    from dcnr import _lib
    batches = [make_batch(gen, CFG2_B, dev)[:4] for _ in range(4)]
    out = torch.empty((CFG2_B, D), dtype=torch.float32, device=dev)
    for k in range(3):
        model.gather_cross(*batches[k % 4], out=out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(iters):
        model.gather_cross(*batches[k % 4], out=out)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    _lib.profile_enable(True)
    _lib.profile_collect()
    for k in range(iters):
        model.gather_cross(*batches[k % 4], out=out)
    _lib.profile_enable(False)
    ms, cnt = _lib.profile_collect()["gather_cross"]
    t_launch = ms / cnt / 1e3
    achieved = CFG2_BYTES * CFG2_B / t_launch / 1e9
    traffic = pmc_traffic("gather_cross_cfg2")
    return {"workload": "BASELINE configs[1]: embedding gather + x0 + 3-layer cross forward, fp32, "
                        "1M x 32 / 100k x 32 / 12 x 1000 x 32 tables, 8 dense",
            "batch": CFG2_B, "dtype": "f32",
            "pairs_per_sec": world * CFG2_B * iters / wall,
            "kernel_pairs_per_sec": CFG2_B / t_launch,
            "roofline": {"bound": "hbm", "kernel": "gather_cross_v4_kernel (dcnr_gather_cross)",
                         "achieved": achieved, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                         "frac": achieved / (PEAK_HBM / 1e9),
                         "traffic": traffic,
                         # the 12 categorical tables (1.5 MB) stay in L2: the
                         # HBM-side rate is the PMC bytes over the same time
                         "traffic_rate_gbs": traffic / t_launch / 1e9 if traffic else None,
                         "bytes_per_sample": CFG2_BYTES, "avg_launch_ms": ms / cnt}}


def bench_cfg5(dev, iters, cpu):
    """BASELINE configs[4]: cosine top-k over 1M hotel vectors (d=64) feeding
    the DCN-R ranking batch (dcnr.serving.RankingPipeline; the item table of a
    DCN-R with n_items = 1M, emb_dim = 64).  Top-k per-launch time from HIP
    events (class knn); end-to-end request latency = candidates of Q=32
    positive hotels (one batched top-11) -> union -> ranking batch -> eval
    forward -> sort -> MMR (lambda 0.7, top 20), host syncs included."""
    import dcnr
    from dcnr import _lib
    torch.manual_seed(5)
    n_items = 1_000_000
    m = dcnr.DCN_RecSys(1_000_000, n_items, CFG["cat_dims"], CFG["n_num"],
                        dict(CFG["params"], emb_dim=64), precision="bf16").to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(7)
    item_cat = torch.randint(0, 1000, (n_items, 12), generator=g, device=dev)
    item_num = torch.rand((n_items, 8), generator=g, device=dev)
    pipe = dcnr.RankingPipeline(m, item_cat, item_num)
    table_bytes = n_items * (64 * 4 + 4)
    out = {"workload": "BASELINE configs[4]: cosine top-11 over 1M x 64 hotel vectors fused into "
                       "a DCN-R ranking batch (emb_dim 64, 12 x 1000 cat, 8 dense, 3 cross, "
                       "4 x 512, bf16 eval)", "k": 11}
    lib = _lib.load()
    ix = pipe.index
    packed_ptr = ix._packed.data_ptr() if ix._packed is not None else None
    for Q in (1, 32, 256):
        q = ix._table[torch.randint(0, n_items, (Q,), generator=g, device=dev)]
        for _ in range(2):
            ix.kneighbors_device(q, 11)
        # per call, back to back on one stream (a serving loop's rate): the
        # C entry point with its buffers allocated once, HIP events around
        # `iters` calls
        idx = torch.empty((Q, 11), dtype=torch.int64, device=dev)
        dst = torch.empty((Q, 11), dtype=torch.float32, device=dev)
        nb = int(lib.dcnr_cosine_topk_workspace_size(n_items, Q, 11))
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        call = (ix._table.data_ptr(), ix._inv.data_ptr(), packed_ptr, n_items, 64, q.data_ptr(), Q, 11,
                idx.data_ptr(), dst.data_ptr(), ws.data_ptr(), nb, _lib.stream_ptr(dev))
        _lib.check(lib.dcnr_cosine_topk_packed(*call), "dcnr_cosine_topk")
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(iters):
            lib.dcnr_cosine_topk_packed(*call)
        ev1.record()
        ev1.synchronize()
        _lib.check(lib.dcnr_cosine_topk_packed(*call), "dcnr_cosine_topk")
        t = ev0.elapsed_time(ev1) / 1e3 / iters
        # ... and each call alone between two events (class knn: the events'
        # own cost included)
        _lib.profile_enable(True)
        _lib.profile_collect()
        for _ in range(iters):
            ix.kneighbors_device(q, 11)
        _lib.profile_enable(False)
        ms, cnt = _lib.profile_collect()["knn"]
        out[f"topk_q{Q}_event_bracketed_us"] = ms / cnt * 1e3
        out[f"topk_q{Q}_us"] = t * 1e6
        out[f"topk_q{Q}_queries_per_sec"] = Q / t
        # the batched path (scan v4, every Q here) streams the fit-time bf16
        # copy of the normalised table (2 B / element, dcnr_cosine_pack_rows)
        # once per call; the scoring is 2 N Q d FLOP (bf16 MFMA coarse pass +
        # exact fp32 rescoring of the few admitted rows -- their row gathers,
        # ~Q x 400 x 260 B, are not counted as algorithmic bytes): the MFMA
        # time is below the HBM time, so HBM bounds the call.
        # fp32_mfma_floor_us: the same FLOP at the fp32 MFMA peak (the bound
        # of an all-fp32 scan)
        flop = 2.0 * n_items * Q * 64
        packed = pipe.index._packed is not None
        nbytes = n_items * 64 * 2 if packed else table_bytes
        knn_pmc = {}
        try:
            knn_pmc = json.load(open(os.path.join(ROOT, "profiles", "knn_pmc_traffic.json")))
        except Exception:
            pass
        out["roofline" if Q == 1 else f"roofline_q{Q}"] = {
            "traffic": knn_pmc.get(f"topk_q{Q}"),   # PMC HBM bytes per call (whole chain)
            "bound": "hbm", "kernel": "bound5 (+ merge) + scan4 (bf16 MFMA%s) + rescore (dcnr_cosine_topk, Q=%d)"
            % (" over the fit-time bf16 copy" if packed else "", Q),
            "achieved": nbytes / t / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
            "frac": nbytes / t / PEAK_HBM, "bytes_per_call": nbytes,
            "floor_us": max(nbytes / PEAK_HBM, flop / PEAK_BF16) * 1e6,
            "flop_per_call": flop, "fp32_mfma_floor_us": flop / 157.3e12 * 1e6}
    users = torch.randint(0, 1_000_000, (iters,), generator=g, device=dev).tolist()
    pos = [torch.randint(0, n_items, (32,), generator=g, device=dev) for _ in range(iters)]
    for k in range(2):
        pipe.recommend(users[k], pos[k], lambda_param=0.7)
    torch.cuda.synchronize()
    n_scored = sum(pipe.candidates(p).numel() for p in pos)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(iters):
        pipe.recommend(users[k], pos[k], lambda_param=0.7)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out["request_ms"] = el / iters * 1e3
    out["requests_per_sec"] = iters / el
    out["candidates_per_request"] = n_scored / iters
    out["scored_pairs_per_sec"] = n_scored / el
    if cpu:
        try:
            from sklearn.neighbors import NearestNeighbors as SkNN
            tab = pipe.index._table.cpu().numpy()
            nn = SkNN(n_neighbors=11, metric="cosine", algorithm="brute").fit(tab)
            t0 = time.perf_counter()
            for j in range(3):
                nn.kneighbors(tab[j:j + 1], n_neighbors=11)
            cpu_t = (time.perf_counter() - t0) / 3
            out["cpu_baseline_topk"] = {"value": 1.0 / cpu_t, "unit": "queries/s",
                                        "cores": int(os.environ.get("OMP_NUM_THREADS",
                                                                    os.cpu_count() or 1)),
                                        "kind": "reference",
                                        "sample": "sklearn NearestNeighbors(cosine, brute)"
                                                  ".kneighbors, 3 single queries on the same "
                                                  "1M x 64 table (main.py:268-270, 200)"}
        except Exception as e:   # sklearn absent: report nothing rather than a fake number
            out["cpu_baseline_topk"] = {"error": repr(e)}
    del pipe, m
    torch.cuda.empty_cache()
    return out


def bench_cfg5_sharded(dev, iters, world):
    """SURVEY 8(e) cfg5 at N > 1: the 1M x 64 index row-sharded over the ranks
    (dcnr.ShardedNearestNeighbors: each rank scans 1M/world rows, all-gather
    of the world*k candidates, dcnr_topk_merge), barrier-bracketed, max over
    ranks; the same answer as the single index (tests/test_knn_sharded_gpu.py)."""
    import dcnr
    n, d = 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(11)
    tab = torch.randn((n, d), generator=g, device=dev)
    nn = dcnr.ShardedNearestNeighbors(n_neighbors=11, device=dev).fit(tab)
    del tab
    out = {"workload": f"cosine top-11 over 1M x 64, rows sharded over {world} ranks "
                       f"({nn.hi - nn.lo} rows on rank 0), all-gather + merge"}
    for Q in (1, 32, 256):
        q = torch.randn((Q, d), generator=g, device=dev)
        for _ in range(2):
            nn.kneighbors_device(q, 11)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            nn.kneighbors_device(q, 11)
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        t = float(el.item()) / iters
        out[f"topk_q{Q}_us"] = t * 1e6
        out[f"topk_q{Q}_queries_per_sec"] = Q / t
    del nn
    torch.cuda.empty_cache()
    return out


def bench_fp32(B, dev, pool, world, steps=5, warmup=2):
    """The fp32 parity mode (f32 MFMA GEMMs, fp32 activations: the path pinned
    element-wise to the reference's fixtures) at the same workload: train
    steps per second on the same batches."""
    import dcnr
    torch.manual_seed(42)
    m = dcnr.DCN_RecSys(CFG["n_users"], CFG["n_items"], CFG["cat_dims"], CFG["n_num"],
                        dict(CFG["params"]), precision="fp32").to(dev)
    tr = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4, optimizer_name="AdamW")
    for k in range(warmup):
        tr.step(*pool[k % len(pool)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        tr.step(*pool[(warmup + k) % len(pool)])
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    del tr, m
    torch.cuda.empty_cache()
    return {"samples_per_sec": world * B * steps / el, "ms_per_step": el / steps * 1e3,
            "steps": steps, "dtype": "f32"}


def measured_peaks(dev, iters=10):
    """the box's achievable peaks next to the spec ones -- a
    1 GiB device-to-device stream copy (read + write bytes / time) and a
    large bf16 GEMM through torch (hipBLASLt), both with HIP events."""
    n = 1 << 28   # 1 GiB of fp32
    src = torch.empty(n, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    for _ in range(2):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    copy_gbs = 2 * 4 * n * iters / (e0.elapsed_time(e1) / 1e3) / 1e9
    del src, dst
    m = 8192
    a = torch.randn((m, m), device=dev).to(torch.bfloat16)
    b = torch.randn((m, m), device=dev).to(torch.bfloat16)
    for _ in range(2):
        torch.mm(a, b)
    e0.record()
    for _ in range(iters):
        torch.mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    gemm_tf = 2 * m ** 3 * iters / (e0.elapsed_time(e1) / 1e3) / 1e12
    del a, b
    torch.cuda.empty_cache()
    return {"copy_gbs": copy_gbs, "copy": "1 GiB fp32 device copy (torch), read + write bytes",
            "bf16_gemm_tflops": gemm_tf, "gemm": "8192^3 bf16 torch.mm (hipBLASLt)"}


def pmc_traffic(kernel_class):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(kernel_class)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--pool", type=int, default=0,
                    help="distinct synthetic batches (default: warmup + steps, a fresh batch "
                         "every step)")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 parity-mode line")
    ap.add_argument("--eval-steps", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-serving", action="store_true", help="skip the configs[4] top-k leg")
    ap.add_argument("--no-zipf", action="store_true", help="skip the Zipf(1.05)-id train line")
    ap.add_argument("--exchange", default="dense", choices=["dense", "sparse"],
                    help="N>1 gradient exchange: dense = the dense parameters' all-reduce "
                         "started inside the backward + reduce-scatter / sharded AdamW / "
                         "all-gather of the tables; sparse = owner-bucketed user-table rows + "
                         "all-reduce of the rest")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # --gpus N without a launcher: start N ranks (one process per GPU)
        # under torch.distributed.run before anything touches the GPU, and
        # exit with the launcher's status
        import socket
        import subprocess
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
               f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.run(cmd).returncode)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DCNR_BENCH_REHEARSE=1: every rank on cuda:0 over gloo, to exercise the
    # N>1 code path (exchange, max-over-ranks timing, sharded index, the JSON
    # line) on a one-GPU box; its numbers are not a scaling measurement
    rehearse = os.environ.get("DCNR_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    # N > 1: which backend the ranks run and which device each one drives,
    # so a driver SCALE line shows whether RCCL saw N distinct GPUs
    ranks_info = None
    if world > 1:
        props = torch.cuda.get_device_properties(dev)
        mine = {"rank": rank, "local_rank": local, "device": f"cuda:{local}", "name": props.name,
                "pci_bus_id": getattr(props, "pci_bus_id", None),
                "uuid": str(getattr(props, "uuid", "")) or None}
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, mine)
    import dcnr
    from dcnr import _lib

    B = args.batch
    torch.manual_seed(42)
    model = dcnr.DCN_RecSys(CFG["n_users"], CFG["n_items"], CFG["cat_dims"], CFG["n_num"],
                            dict(CFG["params"]), precision=args.precision).to(dev)
    trainer = dcnr.FusedTrainer(model, lr=1e-3, weight_decay=1e-4, optimizer_name="AdamW",
                                exchange=args.exchange)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 * rank)
    npool = args.pool if args.pool > 0 else args.warmup + args.steps
    pool = [make_batch(gen, B, dev) for _ in range(npool)]

    for k in range(args.warmup):
        trainer.step(*pool[k % len(pool)])
    trainer.check_indices()
    off = args.warmup   # timed steps use batches no warmup step saw

    def timed(instrumented):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if instrumented:
            _lib.profile_enable(instrumented)
            _lib.profile_collect()
        t0 = time.perf_counter()
        for k in range(args.steps):
            last = trainer.step(*pool[(off + k) % len(pool)])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        prof = None
        if instrumented:
            _lib.profile_enable(False)
            prof = _lib.profile_collect(with_bytes=True)
        el_t = torch.tensor([el], device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
        return float(el_t.item()), prof, last

    # timed region: K plain steps (the reported value)
    el, _, loss = timed(False)
    # the same K steps again with every libdcnr launch bracketed by HIP events
    # on its stream (per-kernel-class durations for the roofline); the events
    # serialise launches, so this pass is not the throughput number
    el_prof, prof, _ = timed(True)
    # and once more timing only the weight-gradient GEMMs, in place on their
    # side stream under the dX chain (profile mode 2): their concurrent wall
    # time, the contention the alone-priced table above does not show
    _, prof_dw, _ = timed(2) if args.precision == "bf16" else (None, None, None)
    trainer.check_indices()
    final_loss = float(loss.item())
    # N > 1: the same K steps with the other table exchange on the same
    # trainer (both are ZeRO-1: the moments are sharded the same way), so the
    # line reports both (DESIGN.md section 6 has the per-rank byte model)
    other_exchange = None
    if world > 1 and trainer.shard:
        keep = trainer.exchange
        trainer.exchange = "sparse" if keep == "dense" else "dense"
        try:
            el_o, _, _ = timed(False)
            other_exchange = {"exchange": trainer.exchange, "ms_per_step": el_o / args.steps * 1e3,
                              "value": world * B * args.steps / el_o}
            if trainer.exchange == "sparse" and trainer.last_exchange:
                other_exchange["last_step"] = trainer.last_exchange
        except ValueError as e:   # layout not shard-aligned
            other_exchange = {"exchange": trainer.exchange, "error": str(e)}
        trainer.exchange = keep
    # N > 1: the time each exchange adds after the backward's last kernel
    # (exchange + AdamW, CUDA events around them: VERDICT r04 item 7), max
    # over ranks, from K more steps per exchange outside the timed region
    exchange_window = None
    if world > 1:
        exchange_window = {}
        keep = trainer.exchange
        for ex in ((keep, "sparse" if keep == "dense" else "dense") if trainer.shard else (keep,)):
            trainer.exchange = ex
            trainer.step_events = []
            try:
                timed(False)
                w = torch.tensor([trainer.exchange_window_ms()], device=dev, dtype=torch.float64)
                dist.all_reduce(w, op=dist.ReduceOp.MAX)
                exchange_window[ex + "_ms"] = float(w.item())
            except ValueError:
                pass
            trainer.step_events = None
        trainer.exchange = keep

    # scored pairs/s: eval-mode forward (running-stat BN, no dropout) per GPU
    model.eval()
    with torch.no_grad():
        for k in range(2):
            model(*pool[k % len(pool)][:4])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for k in range(args.eval_steps):
            model(*pool[k % len(pool)][:4])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        ev = torch.tensor([time.perf_counter() - t1], device=dev, dtype=torch.float64)
        # the same eval calls once more with every launch bracketed by HIP
        # events: the library's algorithmic bytes per scored pair and the
        # per-class times of the eval forward (main.py:319-322)
        torch.cuda.synchronize()
        _lib.profile_enable(True)
        _lib.profile_collect()
        for k in range(args.eval_steps):
            model(*pool[k % len(pool)][:4])
        torch.cuda.synchronize()
        _lib.profile_enable(False)
        eprof = _lib.profile_collect(with_bytes=True)
    if world > 1:
        dist.all_reduce(ev, op=dist.ReduceOp.MAX)
    pairs_per_s = world * B * args.eval_steps / float(ev.item())
    n_pairs = B * args.eval_steps
    eval_bytes_pair = sum(v[2] for v in eprof.values() if v[1]) / n_pairs
    eval_gbs = eval_bytes_pair * pairs_per_s / world / 1e9   # per GPU
    eval_tf = EVAL_FLOP_PER_PAIR * pairs_per_s / world / 1e12
    # the fused tower keeps the activations on chip: the eval forward is then
    # MFMA-bound (its bytes per pair are the x0 row, zc and the logit), so the
    # MFMA view is the roofline and the HBM view is reported beside it
    tower = "tower" in eprof and eprof["tower"][1] > 0
    tower_ms = eprof["tower"][0] / args.eval_steps if tower else None
    eval_roof = {
        "bound": "mfma" if tower else "hbm",
        "unit": "TFLOP/s" if tower else "GB/s", "scope": "whole eval forward (every launch), per GPU",
        "achieved": eval_tf if tower else eval_gbs,
        "peak": PEAK_BF16 / 1e12 if tower else PEAK_HBM / 1e9,
        "frac": eval_tf * 1e12 / PEAK_BF16 if tower else eval_gbs * 1e9 / PEAK_HBM,
        "bytes_per_pair": eval_bytes_pair,
        "hbm_view": {"achieved_gbs": eval_gbs, "peak_gbs": PEAK_HBM / 1e9,
                     "frac": eval_gbs * 1e9 / PEAK_HBM},
        "flop_per_pair": EVAL_FLOP_PER_PAIR,
        "mfma_view": {"achieved_tflops": eval_tf, "peak_tflops": PEAK_BF16 / 1e12,
                      "frac": eval_tf * 1e12 / PEAK_BF16},
        "tower_kernel": None if not tower else {
            "us_per_call": tower_ms * 1e3, "samples_per_call": B,
            "achieved_tflops": EVAL_FLOP_PER_PAIR * B / (tower_ms * 1e-3) / 1e12,
            "frac_of_bf16_peak": EVAL_FLOP_PER_PAIR * B / (tower_ms * 1e-3) / PEAK_BF16},
        "by_class": {k: {"ms_per_call": v[0] / args.eval_steps, "launches_per_call":
                         v[1] / args.eval_steps, "bytes_per_pair": v[2] / n_pairs}
                     for k, v in eprof.items() if v[1]},
    }
    zipf = None if args.no_zipf else bench_zipf(trainer, dev, B, world)
    peaks = measured_peaks(dev) if rank == 0 else None
    fp32 = None if args.no_fp32 else bench_fp32(B, dev, pool, world)
    cfg2 = bench_cfg2(model, gen, dev, max(args.steps, 10), world)
    cfg5 = bench_cfg5(dev, 10, world == 1 and rank == 0 and not args.no_cpu_baseline) \
        if not args.no_serving else None
    if cfg5 is not None and world > 1:
        cfg5["sharded_index"] = bench_cfg5_sharded(dev, 10, world)

    if rank == 0:
        samples = world * B * args.steps
        per_step_ms = {k: v[0] / args.steps for k, v in prof.items() if v[1]}
        launches = {k: v[1] / args.steps for k, v in prof.items() if v[1]}
        # every kernel class priced against HBM with the library's per-launch
        # algorithmic bytes (dcnr_profile_collect_bytes); the dominant class
        # (largest time per step among the accounted ones) is `roofline`
        table = {}
        for k, (ms, cnt, nb) in prof.items():
            if not cnt or nb <= 0:
                continue
            t_l = ms / cnt / 1e3
            b_l = nb / cnt
            table[k] = {"ms_per_step": ms / args.steps, "launches_per_step": cnt / args.steps,
                        "avg_launch_ms": ms / cnt, "bytes_per_launch": b_l,
                        "achieved_gbs": b_l / t_l / 1e9, "frac": b_l / t_l / PEAK_HBM,
                        "kernel": CLASS_KERNELS.get(k, k)}
        # `roofline` is the dominant KERNEL: the largest per-step time among
        # the classes that are one kernel function (gemm_fwd / gemm_dx /
        # rowwise mix several kernels and epilogues; they are in the table)
        single = [k for k in table if k in SINGLE_KERNEL_CLASSES]
        dom = max(single, key=lambda k: table[k]["ms_per_step"])
        dt = table[dom]
        roof = {"bound": "hbm", "class": dom, "kernel": dt["kernel"],
                "rule": "largest per-step time among single-kernel classes (roofline_by_class "
                        "lists every class)",
                "achieved": dt["achieved_gbs"], "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                "frac": dt["frac"], "traffic": pmc_traffic(dom),
                "traffic_source": "profiles/pmc_traffic.json (rocprofv3 --pmc passes of the "
                                  "committed profile set r06fin2, not measured in this run)",
                "bytes_per_launch": dt["bytes_per_launch"], "avg_launch_ms": dt["avg_launch_ms"]}
        roof["frac_of_measured_copy"] = dt["achieved_gbs"] / peaks["copy_gbs"]
        if prof_dw and prof_dw.get("gemm_dw", (0, 0, 0))[1] and dom == "gemm_dw":
            c_ms, c_cnt, _ = prof_dw["gemm_dw"]
            roof["concurrent"] = {
                "avg_launch_ms": c_ms / c_cnt, "ms_per_step": c_ms / args.steps,
                "note": "the same launches timed in place on the side stream, overlapping the "
                        "main stream's dX GEMMs and BN passes (profile mode 2)"}
        if dom in GEMM_FLOP:
            flop_launch = GEMM_FLOP[dom] * B * args.steps / prof[dom][1]
            roof["mfma_view"] = {"achieved_tflops": flop_launch / (dt["avg_launch_ms"] / 1e3) / 1e12,
                                 "peak_tflops": PEAK_BF16 / 1e12 if args.precision == "bf16"
                                 else 157.3, "flop_per_launch": flop_launch}
        deep_ms = sum(per_step_ms.get(k, 0.0) for k in GEMM_FLOP)
        deep_flop = sum(GEMM_FLOP.values()) * B
        g_ms, g_cnt, _ = prof["gather_cross"]
        gather_gbs = GATHER_BYTES * B * args.steps / g_cnt / (g_ms / g_cnt / 1e3) / 1e9
        out = {
            "metric": "fwd+bwd samples/sec (DCN-R train step) + scored (user,hotel) pairs/sec",
            "value": samples / el,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "ms_per_step_instrumented": el_prof / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (uniform ids, U[0,1) dense, Bernoulli labels; a distinct batch per "
                    "step, generated on the device before the timed region; weights seed 42, "
                    "torch default init)",
            "config": {"workload": "DCN-R train step: fwd (train BN, dropout 0.6) + BCE + bwd + "
                                   "AdamW (+grad all-reduce), BASELINE configs[2]/[3]",
                       "batch_per_gpu": B, "global_batch": world * B,
                       "tables": "1M x 32 users, 100k x 32 hotels, 12 x 1000 x 32 cat, 8 dense",
                       "deep": "3 cross + 4 x 512 residual", "parallelism": f"dp{world}",
                       "backend": dist.get_backend() if world > 1 else None,
                       "rank_devices": None if world == 1 else
                       [f'{r["device"]} bus {r["pci_bus_id"]}' for r in ranks_info],
                       "exchange": "none" if world == 1 else (
                           "dense params: all-reduce started in the backward (overlapped); "
                           "user/item tables: touched rows all_to_all to the shard owners + "
                           "sharded AdamW + all-gather; categorical tables: all-reduce"
                           if args.exchange == "sparse"
                           else "dense params: all-reduce started in the backward (overlapped); "
                                "tables: reduce-scatter + sharded AdamW + all-gather, "
                                f"pipelined in {trainer.chunks} chunks"),
                       "exchange_chunks": trainer.chunks if world > 1 else None},
            "distributed": None if world == 1 else {
                "backend": dist.get_backend(), "world_size": world, "ranks": ranks_info,
                "distinct_devices": len({(r["pci_bus_id"], r["uuid"], r["local_rank"]) for r in ranks_info})},
            "scored_pairs_per_sec": pairs_per_s,
            "scored_pairs_roofline": eval_roof,
            "other_exchange": other_exchange,
            "exchange_window_after_backward": exchange_window,
            "final_loss": final_loss,
            "roofline": roof,
            "roofline_by_class": table,
            "deep_tower_mfma": {"gemm_ms_per_step": deep_ms, "flop_per_step": deep_flop,
                                "achieved_tflops": deep_flop / (deep_ms / 1e3) / 1e12 if deep_ms else None,
                                "frac_of_bf16_peak": deep_flop / (deep_ms / 1e3) / PEAK_BF16 if deep_ms else None,
                                "step_tflops": deep_flop / (el / args.steps) / 1e12,
                                "frac_of_measured_gemm": deep_flop / (deep_ms / 1e3) / 1e12 /
                                peaks["bf16_gemm_tflops"] if deep_ms else None},
            "fp32_parity_mode": fp32,
            "zipf_ids": zipf,
            "measured_peaks": peaks,
            "roofline_gather": {"bound": "hbm", "kernel": "gather_cross", "achieved": gather_gbs,
                                "peak": PEAK_HBM / 1e9, "unit": "GB/s",
                                "frac": gather_gbs / (PEAK_HBM / 1e9),
                                "bytes_per_sample": GATHER_BYTES, "avg_launch_ms": g_ms / g_cnt},
            "configs1": cfg2,
            "configs4": cfg5,
            "kernel_ms_per_step": per_step_ms,
            "kernel_launches_per_step": launches,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        if rehearse:
            out["rehearsal"] = "DCNR_BENCH_REHEARSE: all ranks on cuda:0 over gloo (not a scaling number)"
        # both halves of BASELINE's metric, restated LAST so that a record
        # keeping only the line's tail still holds them
        tk = eval_roof["tower_kernel"] or {}
        out["summary"] = {
            "train_samples_per_sec": out["value"], "ms_per_step": out["ms_per_step"],
            "scored_pairs_per_sec": pairs_per_s,
            "scored_pairs_frac_of_bf16_peak": eval_roof["mfma_view"]["frac"],
            "tower_kernel_frac_of_bf16_peak": tk.get("frac_of_bf16_peak"),
            "tower_us_per_131072": tk.get("us_per_call", 0) * 131072 / B if tk else None,
            "deep_tower_mfma_frac": out["deep_tower_mfma"]["frac_of_bf16_peak"],
            "gemm_fwd_avg_launch_ms": table.get("gemm_fwd", {}).get("avg_launch_ms"),
            "roofline_frac": roof["frac"], "roofline_class": dom,
            "gather_frac": out["roofline_gather"]["frac"],
            "topk_us": None if cfg5 is None else
            {f"q{Q}": cfg5.get(f"topk_q{Q}_us") for Q in (1, 32, 256)},
            "request_ms": None if cfg5 is None else cfg5.get("request_ms"),
            "cpu_baseline_samples_per_sec": out.get("cpu_baseline", {}).get("value"),
        }
        if exchange_window:
            out["summary"]["exchange_window_ms"] = exchange_window
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
