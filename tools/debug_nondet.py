"""Round-5 debug: run the same train forward/backward twice on one model and
batch (tests/test_embed_bwd_gpu.py's skewed batch) and report which stored
tensors and gradients differ between the two runs."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch
import test_embed_bwd_gpu as T
from dcnr import _lib

dev = torch.device("cuda")
cfg = T._cfg()
m = T._model(cfg, dev, "bf16", keep=os.environ.get("KEEP", "0") == "1")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
batch = T._skewed_batch(cfg, B, dev, seed=6)
runs = []
for r in range(3):
    g, ws = T._fwd_bwd(m, batch, seed=21)
    runs.append(([x.clone() for x in g], ws.clone()))
names = [k for k, _ in m.named_parameters()]
kinds = ["x0", "h", "t1", "t2", "a1", "bn_mean", "bn_invstd", "du", "dt2", "da", "dt1", "G", "dx0", "zc", "xcoef", "sc"]
for r in (1, 2):
    bad = [k for k, a, b in zip(names, runs[0][0], runs[r][0]) if not torch.equal(a, b)]
    print(f"run {r}: grads differing: {bad}")
    for kind in kinds:
        for idx in range(4):
            off = m.workspace_offset(B, _lib.TRAIN, kind, idx)
            if off < 0:
                continue
            nxt = 1 << 20
            a = runs[0][1][off:off + nxt]
            b = runs[r][1][off:off + nxt]
            if not torch.equal(a, b):
                n = int((a != b).sum())
                print(f"  ws {kind}[{idx}] differs in {n} of first {nxt} bytes")
