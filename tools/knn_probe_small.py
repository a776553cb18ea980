"""Per-call time of the cosine top-11 over small tables (the reference's own
hotel counts are in the thousands): python3 tools/knn_probe_small.py"""
import os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import dcnr
from dcnr import _lib
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for N in (3000, 20000, 60000):
    tab = torch.randn((N, 64), generator=g, device=dev)
    nn = dcnr.NearestNeighbors(metric="cosine").fit(tab)
    for Q in (1, 32):
        q = tab[torch.randint(0, N, (Q,), generator=g, device=dev)]
        for _ in range(3): nn.kneighbors_device(q, 11)
        torch.cuda.synchronize()
        _lib.profile_enable(True); _lib.profile_collect()
        for _ in range(20): nn.kneighbors_device(q, 11)
        _lib.profile_enable(False)
        ms, cnt = _lib.profile_collect()["knn"]
        print(f"N={N} Q={Q}: {ms/20*1e3:.1f} us per call")
