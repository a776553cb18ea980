"""Round-5 debug: the same train forward/backward repeated with the caching
allocator's blocks poisoned (random bytes) between runs: which gradients /
logits differ (a read of memory no kernel wrote would show here)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
for p in ("tests", "oracle", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch
import test_embed_bwd_gpu as T
from dcnr.model import run_backward, run_forward
from dcnr.ops import bce_with_logits

dev = torch.device("cuda")
cfg = T._cfg()
m = T._model(cfg, dev, "bf16", keep=False)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
batch = T._skewed_batch(cfg, B, dev, seed=4)
res = []
for r in range(4):
    if r >= 2:   # poison: fill a large block with random bytes and free it
        junk = torch.randint(0, 255, (1 << 30,), dtype=torch.uint8, device=dev)
        del junk
    u, i, c, n, y = batch
    logits, ws = run_forward(m, True, 3, u, i, c, n)
    _, dz = bce_with_logits(logits, y)
    grads = [torch.empty_like(q) for q in m.param_tensors()]
    run_backward(m, u, i, c, n, dz, ws, grads, 3)
    torch.cuda.synchronize()
    res.append((logits.clone(), [g.clone() for g in grads]))
    del ws, grads
names = [k for k, _ in m.named_parameters()]
for r in range(1, 4):
    print(f"run {r}: logits equal {torch.equal(res[0][0], res[r][0])}; grads differing:",
          [k for k, a, b in zip(names, res[0][1], res[r][1]) if not torch.equal(a, b)])
