"""Eval forward (bf16) through the fused deep tower (csrc/tower.hip: the
initial Linear, every ResBlock with running-stat BatchNorm, and the deep head
dot in one persistent launch, activations in registers; main.py:319-322 ->
train.py:155-170 in eval mode).  Checked against the layer-by-layer eval path
of the same library (DCNR_FLAG_KEEP_INTERMEDIATES: one streaming GEMM per
Linear with BN + ReLU (+ residual) in its epilogue, bf16 activations in HBM,
row_dot head) and against the fp64 oracle.

Both paths store the same bf16 activations up to the MFMA's summation order
(the tower permutes each hidden layer's input columns inside a 32-column
k-step so a layer's accumulators are the next layer's operand, and folds the
Linear bias into the BN shift): an fp32 rounding difference flips a bf16
rounding now and then, so the logits agree to ~1e-4 of their scale, not bit
for bit.  The tower is deterministic run to run.

Shapes: the bench layer widths (D=456 -> 16 k-steps, H=512), a batch that is
not a multiple of the 128-sample tile, hidden widths padded to 64 (CFG_ODD:
H=96) and configs[0] (H=128), and a batch past 2^31 bytes of x0 (the launch
runs in chunks of 32-bit buffer offsets).  CFG_WIDE (D > 512) is outside the
tower and keeps the layer-by-layer path with the last GEMM's fused head.
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

# 20 categorical tables of width 32: D = 2*32 + 20*32 + 8 = 712 > 512
CFG_WIDE = dict(n_users=3000, n_items=700, cat_dims={f"c{i}": 1000 for i in range(20)}, n_num=8,
                params=dict(emb_dim=32, hidden_dim=256, n_cross_layers=2, n_res_blocks=2, dropout=0.0))


def _model(cfg, dev):
    import dcnr
    torch.manual_seed(gc.WEIGHT_SEED)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), precision="bf16")
    gc.perturb_state(m, gc.WEIGHT_SEED + 1)
    return m.to(dev).eval()


def _eval_logits(m, inp, dev, keep, tower=None):
    u, i, c, n, _ = inp
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    m.keep_intermediates = keep
    m.fused_tower = (not keep) if tower is None else tower   # the tower at every batch size
    with torch.no_grad():
        z = m(t(u), t(i), t(c), t(n))
    torch.cuda.synchronize()
    return z.double().cpu().numpy().reshape(-1)


def _oracle_check(m, cfg, inp, z, B):
    import dcnr_oracle as orc  # checker only
    sd = {k: v.detach().cpu().double().numpy() for k, v in m.state_dict().items()}
    spec = orc.spec_from_params(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                                dict(cfg["params"]))
    sel = np.arange(0, B, max(1, B // 512))
    u, i, c, n, _ = inp
    zr, _ = orc.forward(sd, spec, u[sel], i[sel], c[sel], n[sel], train=False)
    assert np.linalg.norm(z[sel] - zr) / np.linalg.norm(zr) <= 1e-2


@pytest.mark.parametrize("cfg,B", [(gc.CFG3R, 131072), (gc.CFG3R, 4099), (gc.CFG3R, 1),
                                   (gc.CFG1, 777), (gc.CFG_ODD, 1000), (CFG_WIDE, 3000)])
def test_eval_tower_matches_layer_by_layer(dev, cfg, B):
    m = _model(cfg, dev)
    inp = gc.make_inputs(cfg, B, 5)
    zf = _eval_logits(m, inp, dev, keep=False)
    zk = _eval_logits(m, inp, dev, keep=True)
    scale = max(1.0, float(np.abs(zk).max()))
    err = np.abs(zf - zk) / scale
    rel = np.linalg.norm(zf - zk) / max(np.linalg.norm(zk), 1e-30)
    print(f"tower vs layer-by-layer B={B}: max {err.max():.3e} rel {rel:.3e}")
    assert err.max() < 2e-3 and rel < 2e-4
    assert np.array_equal(_eval_logits(m, inp, dev, keep=False), zf)   # deterministic
    _oracle_check(m, cfg, inp, zf, B)


@pytest.mark.parametrize("bad", ["nan_weight", "inf_bias"])
def test_eval_relu_nan_rule_same_in_both_paths(dev, bad):
    """One ReLU rule for NaN in the fused tower and the layer-by-layer
    epilogues: max over the value's sign-magnitude bits, the
    tower's packed-int16 rule -- a positive NaN (what NaN arithmetic yields
    here) and +inf pass, as torch.relu passes NaN (train.py:117); -inf and a
    negative-signed NaN give 0.  A NaN row of the first block's layer1 weight
    (t1[:, j] NaN for every sample) or an infinite bias: both paths give
    the same NaN pattern and the same finite logits."""
    cfg, B = gc.CFG3R, 4099
    m = _model(cfg, dev)
    with torch.no_grad():
        if bad == "nan_weight":
            m.res_blocks[0].layer1.weight[5].fill_(float("nan"))
        else:
            m.res_blocks[0].layer1.bias[5] = float("-inf")
    inp = gc.make_inputs(cfg, B, 5)
    zf = _eval_logits(m, inp, dev, keep=False)
    zk = _eval_logits(m, inp, dev, keep=True)
    print(f"{bad}: NaN logits tower {np.isnan(zf).mean():.3f} layer-by-layer {np.isnan(zk).mean():.3f}")
    assert np.array_equal(np.isnan(zf), np.isnan(zk))
    ok = np.isfinite(zk)
    if ok.any():
        scale = max(1.0, float(np.abs(zk[ok]).max()))
        assert np.abs(zf[ok] - zk[ok]).max() / scale < 2e-3


def test_eval_tower_chunked_launch(dev):
    """2.4M samples: x0 is 2.2 GB of bf16, past the 32-bit buffer offsets of
    one launch; every chunk's logits must equal scoring the same rows alone."""
    cfg, B = gc.CFG3R, 2_400_000
    m = _model(cfg, dev)
    inp = gc.make_inputs(cfg, B, 9)
    z = _eval_logits(m, inp, dev, keep=False)
    for lo in (0, 2_300_000):   # a slice from each launch chunk, scored alone
        part = tuple(a[lo:lo + 5000] for a in inp)
        assert np.array_equal(_eval_logits(m, part, dev, keep=False), z[lo:lo + 5000])
    assert np.isfinite(z).all()


def test_eval_tower_batch_threshold(dev):
    """Without DCNR_FLAG_FUSED_TOWER the bf16 eval forward launches the fused
    tower from 16384 samples on (dcnr_api.hip TOWER_MIN_B: below it the
    layer-by-layer path is faster) -- counted by the library's per-class
    launch profiler -- and its logits there equal the forced tower's bit
    for bit."""
    from dcnr import _lib
    cfg = gc.CFG3R
    m = _model(cfg, dev)
    for B, want in ((16383, 0), (16384, 1)):
        inp = gc.make_inputs(cfg, B, 13)
        _lib.profile_enable(True)
        _lib.profile_collect()
        try:
            z_default = _eval_logits(m, inp, dev, keep=False, tower=False)
            launches = _lib.profile_collect()["tower"][1]
        finally:
            _lib.profile_enable(False)
        assert launches == want, (B, launches)
        if want:
            assert np.array_equal(z_default, _eval_logits(m, inp, dev, keep=False, tower=True))


@pytest.mark.parametrize("col", ["user", "item", "cat", "neg"])
def test_eval_tower_index_check(dev, col):
    """An out-of-range id in a fused-tower eval call raises IndexError --
    deferred (the tower launch stores the call's error word into the pinned
    ring slot the call reserved: no copy, no event) and with
    check_indices="sync" -- and a clean call afterwards raises nothing."""
    cfg = gc.CFG3R
    m = _model(cfg, dev)
    m.fused_tower = True
    u, i, c, n, _ = gc.make_inputs(cfg, 300, 21)
    u, i, c = u.copy(), i.copy(), c.copy()
    if col == "user":
        u[7] = cfg["n_users"]
    elif col == "item":
        i[290] = cfg["n_items"] + 5
    elif col == "cat":
        c[100, 11] = 1000
    else:
        u[0] = -1
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    with torch.no_grad(), pytest.raises(IndexError):
        m(t(u), t(i), t(c), t(n))
        m.check_index_errors()
    m.check_indices = "sync"
    with torch.no_grad(), pytest.raises(IndexError):
        m(t(u), t(i), t(c), t(n))
    m.check_indices = True
    with torch.no_grad():
        for _ in range(20):   # past the ring's in-flight depth: slots recycle
            m(t(u * 0), t(i * 0), t(c * 0), t(n))
        m.check_index_errors()


def test_eval_tower_other_widths(dev):
    """CFG3R with one categorical table widened to 40 / 35 columns (x0 groups
    no longer at multiples of 32): the tower against the layer-by-layer path,
    run to run, and against the fp64 oracle."""
    for card in (1599, 1224):   # int(sqrt(n)) + 1 = 40 / 35
        cfg = dict(gc.CFG3R)
        cats = dict(cfg["cat_dims"])
        cats["c0"] = card
        cfg["cat_dims"] = cats
        m = _model(cfg, dev)
        B = 20000
        inp = gc.make_inputs(cfg, B, 31)
        zf = _eval_logits(m, inp, dev, keep=False)
        zk = _eval_logits(m, inp, dev, keep=True)
        scale = max(1.0, float(np.abs(zk).max()))
        assert np.abs(zf - zk).max() / scale < 2e-3, card
        assert np.array_equal(_eval_logits(m, inp, dev, keep=False), zf)
        _oracle_check(m, cfg, inp, zf, B)
