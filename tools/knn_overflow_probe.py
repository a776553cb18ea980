"""Top-k latency when every query's admitted list overflows (VERDICT r05
item 5: the exact fallback's cliff), 1M x 64, k = 11: each query's direction
planted on 5000 table rows, so scan v4's list passes V4_CAP for every query
and the exact fallback answers; the same queries on the clean table beside.
  python tools/knn_overflow_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import dcnr  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
N, D = 1_000_000, 64
base = torch.randn((N, D), generator=g, device=dev)
for Q in (1, 4, 16, 256):
    q = torch.randn((Q, D), generator=g, device=dev)
    tab = base.clone()
    per = min(5000, N // Q)
    rows = torch.randperm(N, generator=g, device=dev)[:per * Q].view(Q, per)
    for j in range(Q):
        tab[rows[j]] = q[j]
    for name, t in (("clean", base), ("all-overflow", tab)):
        nn_ = dcnr.NearestNeighbors(metric="cosine").fit(t)
        for _ in range(2):
            d, i = nn_.kneighbors_device(q, 11)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 5
        a.record()
        for _ in range(it):
            d, i = nn_.kneighbors_device(q, 11)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / it * 1e3
        ok = ""
        if name == "all-overflow":
            want = torch.sort(rows, dim=1).values[:, :11]
            ok = f" exact: {bool(torch.equal(i.cpu(), want.cpu()))}"
        print(f"Q={Q:4d} {name:12s} {us:9.1f} us per call{ok}", flush=True)
        del nn_
