"""Timing probe for scan v4 lab builds (tools/knn_lab.sh): Q = 32 and 256
queries over a 1M x 64 table, 10 calls each (results not checked: the lab
ablations compute wrong answers on purpose)."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import dcnr  # noqa: E402
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
tab = torch.randn((1_000_000, 64), generator=g, device=dev)
nn = dcnr.NearestNeighbors(metric="cosine").fit(tab)
for Q in (1, 32, 256):
    q = tab[torch.randint(0, 1_000_000, (Q,), generator=g, device=dev)]
    for _ in range(12):
        nn.kneighbors_device(q, 11)
    torch.cuda.synchronize()
print("ok")
