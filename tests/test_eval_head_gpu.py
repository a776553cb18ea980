"""Eval forward's fused tail (bf16): the last block's GEMM ends in the deep
head dot (no h_R is stored) and every eval GEMM makes its BatchNorm affine
from the running statistics itself (main.py:319-322 -> train.py:155-170 in
eval mode).  Checked against the unfused eval path of the same library
(DCNR_FLAG_KEEP_INTERMEDIATES keeps the bn_eval_finalize launch, the stored
h_R and the row_dot head) and against the fp64 oracle.

Both paths compute the same bf16 activations bit for bit; only the head dot's
summation order differs (per-wave partials summed in a fixed order vs one
wave per row), so the logits agree to fp32 rounding of a 512-term dot.
"""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import golden_common as gc  # noqa: E402

pytestmark = pytest.mark.gpu


def _eval_logits(m, inp, dev, keep):
    u, i, c, n, _ = inp
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    m.keep_intermediates = keep
    with torch.no_grad():
        z = m(t(u), t(i), t(c), t(n))
    torch.cuda.synchronize()
    return z.double().cpu().numpy()


# (600000 rows of 512 bf16 columns: the GEMM runs in two M-chunks of 32-bit
# buffer offsets, each writing its rows of the head partials)
@pytest.mark.parametrize("cfg,B", [(gc.CFG3R, 131072), (gc.CFG3R, 4099), (gc.CFG3R, 600000),
                                   (gc.CFG1, 777), (gc.CFG_ODD, 1000)])
def test_eval_fused_head_matches_unfused(dev, cfg, B):
    import dcnr
    import dcnr_oracle as orc  # checker only
    torch.manual_seed(gc.WEIGHT_SEED)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), precision="bf16")
    gc.perturb_state(m, gc.WEIGHT_SEED + 1)
    m = m.to(dev).eval()
    inp = gc.make_inputs(cfg, B, 5)
    zf = _eval_logits(m, inp, dev, keep=False)
    zk = _eval_logits(m, inp, dev, keep=True)
    scale = np.maximum(np.abs(zk), 1.0)
    assert np.max(np.abs(zf - zk) / scale) < 2e-6
    assert np.array_equal(_eval_logits(m, inp, dev, keep=False), zf)   # deterministic
    # and against the fp64 oracle on a sample (bf16 storage of activations)
    sd = {k: v.detach().cpu().double().numpy() for k, v in m.state_dict().items()}
    spec = orc.spec_from_params(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                                dict(cfg["params"]))
    sel = np.arange(0, B, max(1, B // 512))
    u, i, c, n, _ = inp
    zr, _ = orc.forward(sd, spec, u[sel], i[sel], c[sel], n[sel], train=False)
    assert np.linalg.norm(zf[sel] - zr) / np.linalg.norm(zr) <= 1e-2
