"""FusedTrainer without the tables' zero fill: the
backward marks the embedding rows it writes in a byte map
(DCNR_FLAG_ROW_MAP) instead of zeroing 142 MB of table gradients, and
dcnr_adam_step_rows reads unmarked rows' gradients as exactly 0.  The
reference's optimizer (torch.optim.AdamW over dense embedding gradients,
train.py:201-204, 226) moves every row every step; this must stay
bit-identical to the dense-gradient path (dense_table_grads=True)."""
import copy
import ctypes

import numpy as np
import pytest
import torch

from helpers import our_model

pytestmark = pytest.mark.gpu


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def test_adam_step_rows_matches_dense(dev):
    """dcnr_adam_step_rows == dcnr_adam_step on the gradient with the
    unmarked rows zeroed (garbage in those rows is never read), for mapped
    tensors of widths 32 / 3 / 17 and a dense one in the same launch."""
    from dcnr import _lib
    lib = _lib.load()
    g = torch.Generator(device=dev).manual_seed(3)
    shapes = [(5000, 32), (700, 3), (129, 17), (1000, 1)]   # the last: dense
    P = [torch.randn(s, generator=g, device=dev) for s in shapes]
    G = [torch.randn(s, generator=g, device=dev) for s in shapes]
    M = [torch.randn(s, generator=g, device=dev) * 0.1 for s in shapes]
    V = [torch.rand(s, generator=g, device=dev) * 0.01 for s in shapes]
    maps = [(torch.rand(s[0], generator=g, device=dev) < 0.3).to(torch.uint8) for s in shapes[:3]]
    Gd = [x.clone() for x in G]
    for t, mp in enumerate(maps):
        Gd[t][mp == 0] = 0.0
        G[t][mp == 0] = float("nan")            # never read
    P2, M2, V2 = [x.clone() for x in P], [x.clone() for x in M], [x.clone() for x in V]
    n = len(shapes)
    numel = (ctypes.c_int64 * n)(*[x.numel() for x in P])
    for step in (1, 2, 7):
        _lib.check(lib.dcnr_adam_step(n, _ptrs(P), _ptrs(Gd), _ptrs(M), _ptrs(V), numel, 1e-3, 0.9,
                                      0.999, 1e-8, 1e-2, step, 1, _lib.stream_ptr(dev)))
        rm = (ctypes.c_void_p * n)(*[mp.data_ptr() for mp in maps], None)
        rw = (ctypes.c_int32 * n)(*[s[1] for s in shapes[:3]], 1)
        _lib.check(lib.dcnr_adam_step_rows(n, _ptrs(P2), _ptrs(G), _ptrs(M2), _ptrs(V2), numel, rm,
                                           rw, 1e-3, 0.9, 0.999, 1e-8, 1e-2, step, 1,
                                           _lib.stream_ptr(dev)))
    torch.cuda.synchronize()
    for a, b in zip(P + M + V, P2 + M2 + V2):
        assert torch.equal(a, b)
    # a mapped tensor whose size is not a whole number of rows is refused
    bad = (ctypes.c_int32 * n)(33, 3, 17, 1)
    with pytest.raises(ValueError):
        _lib.check(lib.dcnr_adam_step_rows(n, _ptrs(P2), _ptrs(G), _ptrs(M2), _ptrs(V2), numel, rm,
                                           bad, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 1, 1,
                                           _lib.stream_ptr(dev)))


def _trainer_pair(cfg, precision, dev):
    import dcnr
    m1 = our_model(cfg, precision=precision).to(dev)
    m2 = copy.deepcopy(m1)
    t1 = dcnr.FusedTrainer(m1, lr=1e-3, weight_decay=1e-4)              # row map (world 1)
    t2 = dcnr.FusedTrainer(m2, lr=1e-3, weight_decay=1e-4, dense_table_grads=True)
    assert t1.row_map and not t2.row_map
    return m1, m2, t1, t2


def _batch(cfg, B, g, dev, skew):
    nu, ni = cfg["n_users"], cfg["n_items"]
    if skew:   # a hot user, few items: most rows untouched, long runs
        u = torch.where(torch.rand(B, generator=g, device=dev) < 0.4,
                        torch.full((B,), 7, device=dev),
                        torch.randint(0, nu, (B,), generator=g, device=dev))
        i = torch.randint(0, max(1, ni // 50), (B,), generator=g, device=dev)
    else:
        u = torch.randint(0, nu, (B,), generator=g, device=dev)
        i = torch.randint(0, ni, (B,), generator=g, device=dev)
    cd = list(cfg["cat_dims"].values())
    c = torch.stack([torch.randint(0, k, (B,), generator=g, device=dev) for k in cd], 1)
    n = torch.rand((B, cfg["n_num"]), generator=g, device=dev)
    y = (torch.rand(B, generator=g, device=dev) < 0.5).float()
    return u, i, c, n, y


@pytest.mark.parametrize("precision,skew", [("fp32", False), ("bf16", True), ("bf16", False)])
def test_fused_trainer_row_map_bit_identical(dev, precision, skew):
    """3 dropout-0.6 steps: every parameter, moment and BN buffer of the
    row-map trainer equals the dense-gradient trainer's bit for bit, and
    the loss of every step too."""
    cfg = dict(n_users=20000, n_items=3000, cat_dims={"a": 1000, "b": 37, "c": 250}, n_num=5,
               params=dict(emb_dim=32, hidden_dim=128, n_cross_layers=3, n_res_blocks=2,
                           dropout=0.6))
    m1, m2, t1, t2 = _trainer_pair(cfg, precision, dev)
    g = torch.Generator(device=dev).manual_seed(11)
    for s in range(3):
        b = _batch(cfg, 3000, g, dev, skew)
        torch.cuda.manual_seed(100 + s)
        l1 = t1.step(*b)
        torch.cuda.manual_seed(100 + s)
        l2 = t2.step(*b)
        assert torch.equal(l1, l2)
    torch.cuda.synchronize()
    for (k, a), (_, b2) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b2), k
    assert torch.equal(t1.m, t2.m) and torch.equal(t1.v, t2.v)
    # the tables' .grad rows the last step did not touch hold stale values
    # until materialize_table_grads() zeroes them: then every
    # gradient equals the dense path's (zero_grad + backward, train.py:222-225)
    t1.materialize_table_grads()
    torch.cuda.synchronize()
    for (k, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(p1.grad, p2.grad), k


def test_fused_trainer_row_map_bench_model(dev):
    """The bench model (BASELINE configs[2]: 1M x 32 users, 100k x 32 items,
    12 x 1000 x 32, 3 cross, 4 x 512, bf16, dropout 0.6) at B = 131072:
    three steps bit-identical to the dense-gradient path."""
    cfg = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
               n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4,
                                    dropout=0.6))
    m1, m2, t1, t2 = _trainer_pair(cfg, "bf16", dev)
    g = torch.Generator(device=dev).manual_seed(5)
    for s in range(3):
        b = _batch(cfg, 131072, g, dev, False)
        torch.cuda.manual_seed(200 + s)
        t1.step(*b)
        torch.cuda.manual_seed(200 + s)
        t2.step(*b)
    torch.cuda.synchronize()
    assert torch.equal(t1.flat, t2.flat)
    assert torch.equal(t1.m, t2.m) and torch.equal(t1.v, t2.v)
    for (k, a), (_, b2) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b2), k
