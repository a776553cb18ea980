"""Debug dump: one skewed bf16 step, arrays for a few single-sample user rows."""
import sys
import numpy as np
import torch
sys.path[:0] = ["tests", "tests/golden", "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd", "oracle"]
import test_embed_bwd_gpu as t
from dcnr import _lib
dev = torch.device("cuda:0")
cfg = t._cfg()
B = 65536
m = t._model(cfg, dev, "bf16")
batch = t._skewed_batch(cfg, B, dev)
grads, ws = t._fwd_bwd(m, batch, seed=77)
gd = dict(zip([k for k, _ in m.named_parameters()], grads))
D = m._dims["input_dim"]; Dp = (D + 7) // 8 * 8; Dq = (Dp + 31) // 32 * 32
L = 3; H = 256
off = m.workspace_offset(B, _lib.TRAIN, "dx0", 0)
X = ws[off:off + B * Dq * 4].view(torch.float32).view(B, Dq)[:, :D].cpu().numpy()
off = m.workspace_offset(B, _lib.TRAIN, "xcoef", 0)
Cf = ws[off:off + B * 4 * 4].view(torch.float32).view(B, 4).cpu().numpy()
sd = m.state_dict()
V = np.stack([sd[f"cross_network.{l}.w.weight"][0].cpu().numpy() for l in range(L)] + [sd["final_linear.weight"][0, H:].cpu().numpy()])
u = batch[0].cpu().numpy()
g = gd["user_embedding.weight"].cpu().numpy()
np.savez("gpurun_out/dbg_emb.npz", X=X[:, :32], Cf=Cf, V=V[:, :32], u=u, g=g[:64])
print("saved")
