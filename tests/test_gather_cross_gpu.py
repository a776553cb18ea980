"""GPU parity of dcnr_gather_cross (BASELINE configs[1]: embedding gathers +
x0 concat + the cross network, train.py:156-159 and 166-168) against the fp64
oracle (oracle/dcnr_oracle.py gather_x0 / cross_layer).

Tolerances: x0 is a copy, so it must be bit-exact in fp32; cross_out
|d| <= 1e-4 * max(|ref|, 1) element-wise vs fp64 (the north_star's fp32 bar).
Both kernel variants are covered: the 16-byte-lane kernel (every table width
and n_num a multiple of 4: CFG1, CFG3R, the full configs[1] size) and the
general 4-byte-lane kernel (odd widths: CFG_ODD, RANDOM_CFGS[0]).
"""
import numpy as np
import pytest
import torch

import dcnr_oracle as orc
import golden_common as gc
from helpers import np_state, our_model, spec_of, to_dev

pytestmark = pytest.mark.gpu

CFG_MIXED = dict(n_users=500, n_items=300, cat_dims={"a": 5, "b": 200, "c": 1000}, n_num=2,
                 params=dict(emb_dim=16, hidden_dim=160, n_cross_layers=1, n_res_blocks=1,
                             dropout=0.0))
CFG2 = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
            n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4,
                                 dropout=0.6))


def oracle_cross(sd, spec, cfg, u, i, c, n):
    x = orc.gather_x0(sd, spec, u, i, c, n, dt=np.float64)
    for l in range(cfg["params"]["n_cross_layers"]):
        x, _ = orc.cross_layer(x, sd[f"cross_network.{l}.w.weight"][0], sd[f"cross_network.{l}.b"])
    return x


def cross_err(got, ref):
    return float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0))) if ref.size else 0.0


@pytest.mark.parametrize("name,cfg", [("cfg1", gc.CFG1), ("cfg3r", gc.CFG3R), ("odd", gc.CFG_ODD),
                                      ("mixed", CFG_MIXED)])
@pytest.mark.parametrize("B", [1, 37, 300, 4099])
def test_gather_cross_vs_oracle(dev, name, cfg, B):
    m = our_model(cfg).to(dev)
    sd = np_state(m)
    sd32 = {k: v.astype(np.float32) for k, v in sd.items()}
    spec = spec_of(cfg)
    u, i, c, n, _ = gc.make_inputs(cfg, B, 11 + B)
    x0, cross = m.gather_cross(*to_dev(dev, u, i, c, n), return_x0=True)
    x0_ref = orc.gather_x0(sd32, spec, u, i, c, n, dt=np.float32)
    assert x0.shape == x0_ref.shape == cross.shape
    np.testing.assert_array_equal(x0.cpu().numpy(), x0_ref)       # bit-exact gather
    ref = oracle_cross(sd, spec, cfg, u, i, c, n)
    assert cross_err(cross.cpu().double().numpy(), ref) <= 1e-4
    # cross_out alone (no x0 stores) is the same
    cross2 = m.gather_cross(*to_dev(dev, u, i, c, n))
    assert torch.equal(cross, cross2)


def test_gather_cross_empty_and_oob(dev):
    import dcnr
    cfg = gc.CFG1
    torch.manual_seed(0)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), check_indices=True).to(dev)
    u, i, c, n, _ = gc.make_inputs(cfg, 0, 1)
    assert m.gather_cross(*to_dev(dev, u, i, c, n)).shape == (0, orc.input_dim(16, [250] * 8, 4))
    u, i, c, n, _ = gc.make_inputs(cfg, 64, 2)
    c = c.copy()
    c[17, 5] = 250      # one past the end of cat table 5
    with pytest.raises(IndexError):
        m.gather_cross(*to_dev(dev, u, i, c, n))
        m.check_index_errors()
    c[17, 5] = -1
    m.check_indices = "sync"
    with pytest.raises(IndexError):
        m.gather_cross(*to_dev(dev, u, i, c, n))
    c[17, 5] = 3
    m.gather_cross(*to_dev(dev, u, i, c, n))


def test_gather_cross_full_size_cfg2(dev):
    """BASELINE configs[1] at full size: 1M x 32 users, 100k x 32 hotels,
    12 x 1000 x 32 categorical, 8 dense, 3 cross, B = 65536.  Every row of x0
    is checked bit-exact and every row of cross_out against fp64."""
    import dcnr
    cfg = CFG2
    torch.manual_seed(42)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]))
    gc.perturb_state(m, 3)
    m = m.to(dev)
    B = 65536
    u, i, c, n, _ = gc.make_inputs(cfg, B, 21)
    x0, cross = m.gather_cross(*to_dev(dev, u, i, c, n), return_x0=True)
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    spec = spec_of(cfg)
    x0_ref = orc.gather_x0(sd, spec, u, i, c, n, dt=np.float32)
    np.testing.assert_array_equal(x0.cpu().numpy(), x0_ref)
    sd64 = {k: v.astype(np.float64) for k, v in sd.items()}
    ref = oracle_cross(sd64, spec, cfg, u, i, c, n)
    assert cross_err(cross.cpu().double().numpy(), ref) <= 1e-4
    # the fused train/eval path consumes the same front: eval logits of this
    # model match the oracle on a sample of rows
    m.eval()
    with torch.no_grad():
        z = m(*to_dev(dev, u, i, c, n)).cpu().double().numpy()
    rows = np.random.default_rng(1).choice(B, 64, replace=False)
    zr, _ = orc.forward(sd64, spec, u[rows], i[rows], c[rows], n[rows], train=False)
    assert float(np.max(np.abs(z[rows] - zr) / np.maximum(np.abs(zr), 1.0))) <= 1e-4
