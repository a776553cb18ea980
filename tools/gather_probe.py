"""Gather/cross front timing probe: the per-launch time of the gather_cross
class (libdcnr's HIP-event profiling) in the bench model's train forward
(x0 bf16 + zc + the cross backward's per-sample scalars) and eval forward
(x0 bf16 + zc), B = 131072, plus the whole train forward.
  python tools/gather_probe.py            (DCNR_LIB=... selects a lab build)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import golden_common as gc  # noqa: E402
import dcnr  # noqa: E402
from dcnr import _lib  # noqa: E402
from dcnr.model import run_forward  # noqa: E402

dev = torch.device("cuda:0")
cfg = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{i}": 1000 for i in range(12)}, n_num=8,
           params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4, dropout=0.6))
torch.manual_seed(42)
m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"], dict(cfg["params"]),
                    precision="bf16").to(dev)
B = 131072
ins = [[torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in gc.make_inputs(cfg, B, s)[:4]]
       for s in range(4)]
D = 456
for train in (True, False):
    m.train(train)
    ws = None
    with torch.no_grad():
        for k in range(4):
            _, ws = run_forward(m, train, 1 + k, *ins[k % 4], ws=ws)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 30
        a.record()
        for k in range(it):
            _, ws = run_forward(m, train, 1 + k, *ins[k % 4], ws=ws)
        b.record()
        torch.cuda.synchronize()
        call_us = a.elapsed_time(b) / it * 1e3
        _lib.profile_enable(True)
        _lib.profile_collect()
        for k in range(it):
            _, ws = run_forward(m, train, 1 + k, *ins[k % 4], ws=ws)
        _lib.profile_enable(False)
        prof = _lib.profile_collect(with_bytes=True)
    ms, cnt, nb = prof["gather_cross"]
    us = ms / cnt * 1e3
    per = nb / cnt / B
    print(f"{'train' if train else 'eval '} gather_cross {us:7.1f} us/launch  {per:6.0f} B/sample  "
          f"{per * B / us / 1e3:7.0f} GB/s   forward call {call_us:7.1f} us", flush=True)
