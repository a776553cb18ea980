"""Lab: which stage of the train step differs run to run with gemm_wsp in the
forward (tests/test_embed_bwd_gpu.py's flaky pair, same config and batch).
Prints, per repeat, the stored tensors and gradients that differ from the
first run.  python tools/lab/debug_wsp2.py [repeats]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import dcnr  # noqa: E402
from dcnr import _lib  # noqa: E402
from dcnr.model import run_backward, run_forward  # noqa: E402
from dcnr.ops import bce_with_logits  # noqa: E402

dev = torch.device("cuda:0")
cfg = dict(n_users=200_000, n_items=5000, cat_dims={f"c{k}": 1000 for k in range(12)}, n_num=8,
           params=dict(emb_dim=32, hidden_dim=256, n_cross_layers=3, n_res_blocks=2, dropout=0.0))
torch.manual_seed(11)
m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"], dict(cfg["params"]),
                    precision="bf16").to(dev).train()
m.keep_intermediates = False
B = 32768
rng = np.random.default_rng(6)
u = rng.integers(0, cfg["n_users"], B)
u[rng.random(B) < 0.4] = 7
it = np.minimum((cfg["n_items"] * rng.random(B) ** 4).astype(np.int64), cfg["n_items"] - 1)
c = np.stack([rng.integers(0, 1000, B) for _ in range(12)], 1)
c[:, 0] = 5
n = rng.random((B, 8), dtype=np.float32)
y = (rng.random(B) < 0.5).astype(np.float32)
T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
batch = (T(u, torch.int64), T(it, torch.int64), T(c, torch.int64), T(n, torch.float32), T(y, torch.float32))
names = [k for k, _ in m.named_parameters()]
# (kind, index, bytes): whole tensors
kinds = [("x0", 0, B * 456 * 2), ("h", 0, B * 256 * 2), ("t1", 0, B * 256 * 2), ("bn_mean", 0, 256 * 4),
         ("sc", 0, B * 7 * 4), ("dx0", 0, B * 456 * 4), ("xcoef", 0, B * 4 * 4)]


def run():
    uu, ii, cc, nn_, yy = batch
    logits, ws = run_forward(m, True, 21, uu, ii, cc, nn_)
    torch.cuda.synchronize()
    stored = {}
    for k, idx, nb in kinds[:5]:
        off = m.workspace_offset(B, _lib.TRAIN, k, idx)
        if off >= 0:
            stored[k] = ws[off:off + nb].clone()
    _, dz = bce_with_logits(logits, yy)
    grads = [torch.empty_like(q) for q in m.param_tensors()]
    run_backward(m, uu, ii, cc, nn_, dz, ws, grads, 21, False)
    torch.cuda.synchronize()
    for k, idx, nb in kinds[5:]:
        off = m.workspace_offset(B, _lib.TRAIN, k, idx)
        if off >= 0:
            stored[k] = ws[off:off + nb].clone()
    return logits.clone(), stored, grads


ref = run()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
bad_any = False
for r in range(reps):
    lg, st, gr = run()
    diff = []
    if not torch.equal(lg, ref[0]):
        diff.append("logits")
    for k in st:
        if not torch.equal(st[k], ref[1][k]):
            nz = (st[k] != ref[1][k]).nonzero().flatten()
            diff.append(f"{k}[{nz.numel()} bytes from byte {int(nz[0])}]")
            if k == "h":   # bf16 [B][256]: rows, row within its 32-row tile, column waves
                e = torch.unique(nz // 2)
                rows = torch.unique(e // 256).tolist()
                print(f"   h rows {rows} (row % 32: {sorted({r % 32 for r in rows})}, tile {sorted({r // 32 for r in rows})}), "
                      f"column waves {sorted({int(c) // 64 for c in (e % 256).tolist()})}, {e.numel()} elements", flush=True)
    diff += [nm for nm, a, b in zip(names, gr, ref[2]) if not torch.equal(a, b)]
    bad_any |= bool(diff)
    print(f"rep {r}: {'OK' if not diff else 'DIFF ' + ', '.join(diff[:12])}", flush=True)
print("ALL SAME" if not bad_any else "DIFFERS", os.environ.get("DCNR_LIB", "default lib"))
