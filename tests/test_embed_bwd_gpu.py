"""Deterministic embedding backward (csrc/embed_bwd.hip): the dense
embedding gradients of loss.backward() (reference train.py:156-158, 225;
nn.Embedding with sparse=False, i.e. embedding_dense_backward).

grad_t[r] = sum of dx0[b, off_t:off_t+w_t] over the samples b with id_t[b] == r,
dx0 = deep part + sum_k coef[b][k] V_k (the low-rank cross part).  The library sums each row in a FIXED order: runs of <= 16
samples sequentially in ascending b; longer runs one wave per row, walked in
blocks of 64 entries, slot s of S lane slots taking entries s, s+S, ... of
every block in ascending order, slots added in ascending order.  Runs of
more than HSEG entries are cut at the multiples of HSEG of the global sorted
position (table t's entries sit at t*B ..): each piece is summed as a long
run, the pieces added in order.  ``emulate_table`` restates that order in numpy fp32, so the
gradients are checked BIT-EXACT against it, from the kernels' own deep dx0
and cross coefficients (row = deep sum + sum_k coef sum_k V_k, V = (w_0 ..
w_{L-1}, w_f[H:]), each term rounded twice).  The fp64 recomputation of the deep dx0 and of
the cross coefficients is pinned by tests/test_stages_gpu.py.

Skewed ids exercise both paths: a user id taken by 40 % of the batch, a
Zipf-like item column, a categorical column with one value (a run of B) and
one with two values, uniform columns elsewhere.
"""
import numpy as np
import pytest
import torch

import golden_common as gc

pytestmark = pytest.mark.gpu

SHORT = 16   # embed_bwd.hip LIM
BLK = 64     # embed_bwd.hip emb_runs_long_kernel block of entries
HSEG = 2048  # embed_bwd.hip huge-run segment


def emulate_table(ids, X, Cf, Vt, rows, vec, gbase=0):
    """fp32 gradient of one table in the library's summation order: X the
    table's deep dx0 segments [B][w], Cf the cross coefficients [B][nv], Vt
    the basis restricted to the table's columns [nv][w], gbase the global
    sorted position of the table's first entry."""
    B, w = X.shape
    nv = Cf.shape[1]
    order = np.argsort(ids, kind="stable")
    ks = ids[order]
    heads = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    ends = np.r_[heads[1:], B]
    lens = ends - heads
    g = np.zeros((rows, w), np.float32)

    def combine(deep, cs):   # row = deep + sum_k cs_k V_k, two roundings per term
        out = deep.astype(np.float32)
        for k in range(nv):
            out = (out + (np.float32(cs[..., k:k + 1]) * Vt[k]).astype(np.float32)).astype(np.float32)
        return out

    short = lens <= SHORT
    hs, ls = heads[short], lens[short]
    acc = np.zeros((len(hs), w), np.float32)
    csum = np.zeros((len(hs), nv), np.float32)
    for k in range(SHORT):
        sel = ls > k
        acc[sel] += X[order[hs[sel] + k]]
        csum[sel] += Cf[order[hs[sel] + k]]
    g[ks[hs]] = combine(acc, csum)
    G = w // vec

    def seq(a):   # sequential fp32 sum over axis 0 (0 if empty)
        return np.cumsum(a, axis=0, dtype=np.float32)[-1] if len(a) else np.zeros(a.shape[1], np.float32)

    def piece(ent, cfe, cols):   # one wave's slot-ordered sums of a block walk
        m = len(ent)
        gb = (cols.stop - cols.start) // vec
        S = 64 // gb
        sub = ent[:, cols]
        tot = ctot = None
        for s in range(S):   # slot s: entries s, s+S, ... of every BLK-entry block
            idx = [p + j for p in range(0, m, BLK) for j in range(s, BLK, S) if p + j < m]
            t, ct = seq(sub[idx]), seq(cfe[idx])
            tot = t if tot is None else tot + t
            ctot = ct if ctot is None else ctot + ct
        return tot, ctot

    for h, e in zip(heads[~short], ends[~short]):
        ent = X[order[h:e]]
        cfe = Cf[order[h:e]]
        m = e - h
        # huge runs: pieces cut at the global multiples of HSEG
        cuts = [0]
        if m > HSEG:
            first = (gbase + h) // HSEG * HSEG + HSEG - (gbase + h)
            cuts += list(range(first, m, HSEG))
        cuts.append(m)
        out = np.zeros(w, np.float32)
        for cb in range(0, G, 64):
            cols = slice(cb * vec, (cb + min(64, G - cb)) * vec)
            parts = [piece(ent[a:b], cfe[a:b], cols) for a, b in zip(cuts[:-1], cuts[1:])]
            tot, ctot = parts[0]
            for t, ct in parts[1:]:
                tot, ctot = tot + t, ctot + ct
            out[cols] = _combine_cols(tot, ctot, Vt[:, cols])
        g[ks[h]] = out
    return g


def _combine_cols(deep, cs, Vc):
    out = deep.astype(np.float32)
    for k in range(Vc.shape[0]):
        out = (out + (np.float32(cs[k]) * Vc[k]).astype(np.float32)).astype(np.float32)
    return out


def _tables(m, batch_np, cfg):
    """[(grad name, ids, first x0 column, width)]"""
    u, i, c = batch_np
    names = ["user_embedding.weight", "item_embedding.weight"]
    names += [f"cat_embeddings.{k}.weight" for k in range(c.shape[1])]
    ids = [u, i] + [c[:, k] for k in range(c.shape[1])]
    out, col = [], 0
    for nm, idv in zip(names, ids):
        w = m.state_dict()[nm].shape[1]
        out.append((nm, idv, col, w))
        col += w
    return out


def _check_tables(m, cfg, B, ws, grads, batch_np, vec_expected=None):
    from dcnr import _lib
    gd = dict(zip([k for k, _ in m.named_parameters()], grads))
    sd = m.state_dict()
    D = m._dims["input_dim"]
    Dp = (D + 7) // 8 * 8
    Dq = (Dp + 31) // 32 * 32
    L = cfg["params"]["n_cross_layers"]
    H = cfg["params"]["hidden_dim"]
    off = m.workspace_offset(B, _lib.TRAIN, "dx0", 0)
    X = ws[off:off + B * Dq * 4].view(torch.float32).view(B, Dq)[:, :D].cpu().numpy()
    off = m.workspace_offset(B, _lib.TRAIN, "xcoef", 0)
    Cf = ws[off:off + B * (L + 1) * 4].view(torch.float32).view(B, L + 1).cpu().numpy()
    Vfull = np.stack([sd[f"cross_network.{l}.w.weight"][0].cpu().numpy() for l in range(L)]
                     + [sd["final_linear.weight"][0, H:].cpu().numpy()]).astype(np.float32)
    tabs = _tables(m, batch_np, cfg)
    vec = 4 if all(w % 4 == 0 for _, _, _, w in tabs) and Dq % 4 == 0 else 1
    if vec_expected is not None:
        assert vec == vec_expected
    long_runs = huge_runs = 0
    for t, (name, ids, col, w) in enumerate(tabs):
        rows = sd[name].shape[0]
        ref = emulate_table(ids, X[:, col:col + w], Cf, Vfull[:, col:col + w], rows, vec, t * B)
        got = gd[name].cpu().numpy()
        if not np.array_equal(got, ref):
            bad = np.flatnonzero(np.any(got != ref, axis=1))
            cnt = np.bincount(ids, minlength=rows)
            raise AssertionError((name, np.abs(got - ref).max(), len(bad), bad[:5].tolist(),
                                  cnt[bad[:5]].tolist(), got[bad[0]][:4].tolist(),
                                  ref[bad[0]][:4].tolist()))
        cnt = np.bincount(ids, minlength=rows)
        long_runs += int((cnt > SHORT).sum())
        huge_runs += int((cnt > HSEG).sum())
    return long_runs, huge_runs


def _cfg():
    return dict(n_users=200_000, n_items=5000, cat_dims={f"c{k}": 1000 for k in range(12)},
                n_num=8, params=dict(emb_dim=32, hidden_dim=256, n_cross_layers=3,
                                     n_res_blocks=2, dropout=0.0))


def _skewed_batch(cfg, B, dev, seed=3):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, cfg["n_users"], B)
    u[rng.random(B) < 0.4] = 7
    i = np.minimum((cfg["n_items"] * rng.random(B) ** 4).astype(np.int64), cfg["n_items"] - 1)
    cards = list(cfg["cat_dims"].values())
    c = np.stack([rng.integers(0, n, B) for n in cards], 1)
    c[:, 0] = 5
    c[:, 1] = rng.integers(0, 2, B)
    # runs at the huge-run threshold: HSEG (long kernel), HSEG + 1 and
    # 2 HSEG + 1 entries (pieces)
    c[:, 2] = rng.integers(10, cards[2], B)
    p = rng.permutation(B)
    c[p[:HSEG], 2] = 3
    c[p[HSEG:2 * HSEG + 1], 2] = 4
    c[p[2 * HSEG + 1:4 * HSEG + 2], 2] = 6
    n = rng.random((B, cfg["n_num"]), dtype=np.float32)
    y = (rng.random(B) < 0.5).astype(np.float32)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
    return (t(u, torch.int64), t(i, torch.int64), t(c, torch.int64), t(n, torch.float32),
            t(y, torch.float32))


def _model(cfg, dev, precision="bf16", keep=True):
    import dcnr
    torch.manual_seed(11)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), precision=precision)
    gc.perturb_state(m, 12)
    m = m.to(dev).train()
    m.keep_intermediates = keep
    return m


def _fwd_bwd(m, batch, seed, grads=None, accumulate=False):
    from dcnr.model import run_backward, run_forward
    from dcnr.ops import bce_with_logits
    u, i, c, n, y = batch
    logits, ws = run_forward(m, True, seed, u, i, c, n)
    _, dz = bce_with_logits(logits, y)
    if grads is None:
        grads = [torch.empty_like(q) for q in m.param_tensors()]
    run_backward(m, u, i, c, n, dz, ws, grads, seed, accumulate)
    torch.cuda.synchronize()
    return grads, ws


@pytest.mark.parametrize("precision,B", [("bf16", 65536), ("fp32", 65536), ("bf16", 50003)])
def test_embedding_grads_bit_exact_skewed(dev, precision, B):
    """Every table's gradient equals the fixed-order fp32 emulation from the
    kernels' own deep dx0 and cross coefficients, bit for bit; rows no sample
    references are 0.  B = 50003: tables start off the HSEG segment grid."""
    cfg = _cfg()
    m = _model(cfg, dev, precision)
    batch = _skewed_batch(cfg, B, dev)
    grads, ws = _fwd_bwd(m, batch, seed=77)
    long_runs, huge_runs = _check_tables(m, cfg, B, ws, grads,
                                         [t.cpu().numpy() for t in batch[:3]], 4)
    assert long_runs > 1000 and huge_runs >= 6   # all three paths ran


def test_embedding_grads_bit_exact_odd_widths(dev):
    """CFG_ODD (table widths 24, 2, 5, 2: the scalar-column kernels; 4 cross
    layers), every run long (B >> rows): bit-exact against the emulation."""
    cfg = gc.CFG_ODD
    B = 4096
    m = _model(cfg, dev, "fp32")
    u, i, c, n, y = gc.make_inputs(cfg, B, 5)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
    batch = (t(u, torch.int64), t(i, torch.int64), t(c, torch.int64), t(n, torch.float32),
             t(y, torch.float32))
    grads, ws = _fwd_bwd(m, batch, seed=5)
    _check_tables(m, cfg, B, ws, grads, [u, i, c], 1)


def test_full_size_backward_bit_identical(dev):
    """The bench's step (configs[2] shape, B=131072, bf16, dropout 0.6): two
    backward passes from the same state, batch and dropout seed give
    bit-identical gradients for every parameter."""
    import copy
    cfg = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
               n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3,
                                    n_res_blocks=4, dropout=0.6))
    m = _model(cfg, dev, "bf16", keep=False)
    m2 = copy.deepcopy(m)
    B = 131072
    g = torch.Generator(device=dev).manual_seed(9)
    batch = (torch.randint(0, cfg["n_users"], (B,), device=dev, generator=g),
             torch.randint(0, cfg["n_items"], (B,), device=dev, generator=g),
             torch.randint(0, 1000, (B, 12), device=dev, generator=g),
             torch.rand((B, 8), device=dev, generator=g),
             (torch.rand((B,), device=dev, generator=g) < 0.5).float())
    g1, _ = _fwd_bwd(m, batch, seed=1234)
    g2, _ = _fwd_bwd(m2, batch, seed=1234)
    for k, a, b in zip([k for k, _ in m.named_parameters()], g1, g2):
        assert torch.equal(a, b), k


def test_accumulate_doubles(dev):
    """accumulate=1 adds into the grads: a second identical step accumulated
    onto the first gives exactly twice every gradient (the embedding rows
    included: row = old + fresh sum)."""
    cfg = _cfg()
    m = _model(cfg, dev, "bf16", keep=False)
    batch = _skewed_batch(cfg, 16384, dev, seed=4)
    g1, _ = _fwd_bwd(m, batch, seed=3)
    ref = [x.clone() for x in g1]
    _fwd_bwd(m, batch, seed=3, grads=g1, accumulate=True)
    for k, a, r in zip([k for k, _ in m.named_parameters()], g1, ref):
        assert torch.equal(a, 2 * r), k


def test_side_stream_backward_matches_serial(dev):
    """The bf16 backward runs the weight-gradient GEMMs, their split-K reduces
    and the initial bias column sums on the library's side stream; while
    kernel classes are being timed (profile_enable) the library runs them on
    the caller's stream, in order.  Both give bit-identical gradients for
    every parameter."""
    import copy
    from dcnr import _lib
    cfg = _cfg()
    m = _model(cfg, dev, "bf16", keep=False)
    m2 = copy.deepcopy(m)
    batch = _skewed_batch(cfg, 32768, dev, seed=6)
    g_side, _ = _fwd_bwd(m, batch, seed=21)
    _lib.profile_enable(True)
    try:
        g_serial, _ = _fwd_bwd(m2, batch, seed=21)
    finally:
        _lib.profile_enable(False)
        _lib.profile_collect()
    for k, a, b in zip([k for k, _ in m.named_parameters()], g_side, g_serial):
        assert torch.equal(a, b), k


def test_huge_table_radix_fallback(dev):
    """A user table of more than 2^24 rows (beyond the two-level counting
    sort) takes the stable radix-sort path (emb_keys_kernel + rocPRIM).  The
    batch's user ids are k * MUL + 11 for small ids k: mapped through that
    increasing map, the huge model is the small model (same weights on the
    used rows), the sorted (id, sample) order and the run structure are the
    same, so every gradient must be BIT-identical to the small model's
    counting-sort gradients (the user table's at the mapped rows, zero
    elsewhere) and the logits equal."""
    import dcnr
    cat_dims = {"a": 40, "b": 7}
    params = dict(emb_dim=8, hidden_dim=64, n_cross_layers=2, n_res_blocks=1, dropout=0.0)
    NS, MUL = 3000, 5600
    NB = NS * MUL + 16                       # 16.8 M rows > 2^24
    assert NB > (1 << 24)
    torch.manual_seed(0)
    small = dcnr.DCN_RecSys(NS, 120, cat_dims, 3, params, precision="bf16").to(dev)
    big = dcnr.DCN_RecSys(NB, 120, cat_dims, 3, params, precision="bf16").to(dev)
    rows = torch.arange(NS, device=dev) * MUL + 11
    with torch.no_grad():
        for (k, ps), (_, pb) in zip(small.state_dict().items(), big.state_dict().items()):
            if k == "user_embedding.weight":
                pb.zero_()
                pb[rows] = ps
            else:
                pb.copy_(ps)
    rng = np.random.default_rng(7)
    B = 4096
    u = np.minimum(rng.zipf(1.3, B) - 1, NS - 1)   # long runs (popular users) and short ones
    i = rng.integers(0, 120, B)
    c = np.stack([rng.integers(0, 40, B), rng.integers(0, 7, B)], 1)
    x = rng.random((B, 3), dtype=np.float32)
    y = (rng.random(B) < 0.5).astype(np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    out = []
    for m, uu in ((small, T(u)), (big, T(u) * MUL + 11)):
        m.train()
        z = m(uu, T(i), T(c), T(x))
        loss = dcnr.BCEWithLogitsLoss()(z, T(y))
        loss.backward()
        out.append((z.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    torch.cuda.synchronize()
    (zs, gs), (zb, gb) = out
    assert torch.equal(zs, zb)
    for k, g in gs.items():
        if k == "user_embedding.weight":
            assert torch.equal(gb[k][rows], g), k
            mask = torch.ones(NB, dtype=torch.bool, device=dev)
            mask[rows] = False
            assert gb[k][mask].abs().max().item() == 0.0
        else:
            assert torch.equal(gb[k], g), k
