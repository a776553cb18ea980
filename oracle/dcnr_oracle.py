"""CPU oracle for the DCN-R ranking hot path -- TEST INFRASTRUCTURE ONLY.

This module is a plain-numpy restatement of the reference algorithm, used as
the *checker* in ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``.  Nothing in the product path
(``dcnr`` package, ``libdcnr.so``) imports, calls or links it; the product
path fails loudly when the HIP library is missing.

Parity pinning: this restatement is pinned against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``; checked by
``tests/test_oracle_golden.py``).

Every function cites the reference lines it restates (paths relative to the
reference repository root):

* ``train.py:136-141``  table widths ``int(np.sqrt(n_cat)) + 1`` and input dim
* ``train.py:155-170``  ``DCN_RecSys.forward`` (gathers, concat order, deep
  tower, cross stack, ``cat([deep, cross])``, final linear, squeeze)
* ``train.py:96-99``    ``CrossLayer.forward``: ``x + x*(x.w) + b`` (uses the
  *current* layer input, not x0)
* ``train.py:112-122``  ``ResBlock.forward``: L1 -> BN1 -> ReLU -> Dropout ->
  L2 -> BN2 -> += identity -> ReLU
* ``train.py:206,224``  ``BCEWithLogitsLoss`` (mean reduction)
* ``train.py:201-204,226`` ``torch.optim.AdamW`` / ``Adam`` single step
* ``main.py:268-270,300`` sklearn ``NearestNeighbors(metric='cosine',
  algorithm='brute').kneighbors`` (third party: scikit-learn 1.7.2,
  ``sklearn/metrics/pairwise.py`` cosine_distances and
  ``sklearn/neighbors/_base.py`` ``_kneighbors_reduce_func``: argpartition
  then argsort)
* ``main.py:196-203``   candidate union of _generate_candidates
* ``main.py:325``       stable descending sort of the scored candidates
* ``main.py:133-169``   ``rerank_with_mmr`` (pinned by tests/golden/f8_mmr.npz,
  made by running the reference: tests/golden/make_serving_golden.py)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

BN_EPS = 1e-5          # nn.BatchNorm1d default eps (train.py:106,110)
BN_MOMENTUM = 0.1      # nn.BatchNorm1d default momentum


def cat_width(n_cat: int) -> int:
    """Categorical table width rule, train.py:139-140."""
    return int(np.sqrt(n_cat)) + 1


def input_dim(emb_dim: int, cat_dims: Sequence[int], n_num: int) -> int:
    """train.py:140-141."""
    return emb_dim * 2 + sum(cat_width(n) for n in cat_dims) + n_num


@dataclass
class ModelSpec:
    n_users: int
    n_items: int
    cat_dims: List[int]
    n_num: int
    emb_dim: int
    hidden: int
    n_cross: int
    n_res: int
    dropout: float = 0.0

    @property
    def D(self) -> int:
        return input_dim(self.emb_dim, self.cat_dims, self.n_num)


def spec_from_params(n_users, n_items, cat_dims: Dict[str, int], n_num, params) -> ModelSpec:
    """Mirror of the ctor argument handling at train.py:126-134."""
    return ModelSpec(n_users, n_items, list(cat_dims.values()), n_num,
                     params['emb_dim'], params['hidden_dim'], params['n_cross_layers'],
                     params.get('n_res_blocks', 2), params['dropout'])


# --------------------------------------------------------------------------
# forward
# --------------------------------------------------------------------------
@dataclass
class Cache:
    x0: np.ndarray = None
    h_in: List[np.ndarray] = field(default_factory=list)     # block inputs
    t1: List[np.ndarray] = field(default_factory=list)
    xh1: List[np.ndarray] = field(default_factory=list)
    r1: List[np.ndarray] = field(default_factory=list)
    a1: List[np.ndarray] = field(default_factory=list)
    t2: List[np.ndarray] = field(default_factory=list)
    xh2: List[np.ndarray] = field(default_factory=list)
    u: List[np.ndarray] = field(default_factory=list)
    inv1: List[np.ndarray] = field(default_factory=list)
    inv2: List[np.ndarray] = field(default_factory=list)
    masks: List[Optional[np.ndarray]] = field(default_factory=list)
    h_out: np.ndarray = None
    xs: List[np.ndarray] = field(default_factory=list)        # cross inputs x_l
    ss: List[np.ndarray] = field(default_factory=list)        # s_l = x_l . w_l
    xL: np.ndarray = None
    train: bool = False
    B: int = 0


def _bn(t, p, prefix, train, dt):
    """nn.BatchNorm1d forward (train: biased batch var for normalisation,
    running stats updated with momentum 0.1 and the unbiased var)."""
    g = p[prefix + '.weight'].astype(dt)
    b = p[prefix + '.bias'].astype(dt)
    if train:
        mu = t.mean(axis=0)
        var = t.var(axis=0)  # biased
        n = t.shape[0]
        rm = p[prefix + '.running_mean']
        rv = p[prefix + '.running_var']
        p[prefix + '.running_mean'] = ((1 - BN_MOMENTUM) * rm + BN_MOMENTUM * mu).astype(rm.dtype)
        p[prefix + '.running_var'] = ((1 - BN_MOMENTUM) * rv + BN_MOMENTUM * var * n / (n - 1)).astype(rv.dtype)
        p[prefix + '.num_batches_tracked'] = np.asarray(p[prefix + '.num_batches_tracked']) + 1
    else:
        mu = p[prefix + '.running_mean'].astype(dt)
        var = p[prefix + '.running_var'].astype(dt)
    inv = (1.0 / np.sqrt(var + BN_EPS)).astype(dt)
    xh = (t - mu) * inv
    return xh * g + b, xh, inv


def gather_x0(p, spec: ModelSpec, user, item, cat, num, dt=np.float64):
    """Embedding gathers + concat, train.py:156-159 (bit-exact in fp32)."""
    parts = [p['user_embedding.weight'][user], p['item_embedding.weight'][item]]
    for k in range(len(spec.cat_dims)):
        parts.append(p[f'cat_embeddings.{k}.weight'][cat[:, k]])
    parts.append(num)
    return np.concatenate([np.asarray(a, dtype=dt) for a in parts], axis=1)


def cross_layer(x, w, b):
    """CrossLayer.forward, train.py:96-99: x + x*(x.w) + b."""
    s = x @ w
    return x + x * s[:, None] + b, s


def forward(p: Dict[str, np.ndarray], spec: ModelSpec, user, item, cat, num, train=False,
            dropout_masks: Optional[List[np.ndarray]] = None, dt=np.float64):
    """DCN_RecSys.forward (train.py:155-170).  ``p`` is a dict of numpy
    arrays keyed like the reference state_dict; in train mode the BN running
    statistics in ``p`` are updated in place (as nn.BatchNorm1d does).
    Returns (logits[B], cache)."""
    if train and user.shape[0] == 1:
        raise ValueError("Expected more than 1 value per channel when training")
    c = Cache(train=train, B=user.shape[0])
    W = lambda k: np.asarray(p[k], dtype=dt)
    x0 = gather_x0(p, spec, user, item, cat, num, dt)
    c.x0 = x0
    h = x0 @ W('initial_deep_layer.weight').T + W('initial_deep_layer.bias')
    pdrop = spec.dropout if train else 0.0
    for j in range(spec.n_res):
        pre = f'res_blocks.{j}'
        c.h_in.append(h)
        t1 = h @ W(pre + '.layer1.weight').T + W(pre + '.layer1.bias')
        r1, xh1, inv1 = _bn(t1, p, pre + '.bn1', train, dt)
        a1 = np.maximum(r1, 0)
        m = None
        if pdrop > 0:
            m = dropout_masks[j].astype(dt) / (1.0 - pdrop)
            a1 = a1 * m
        t2 = a1 @ W(pre + '.layer2.weight').T + W(pre + '.layer2.bias')
        r2, xh2, inv2 = _bn(t2, p, pre + '.bn2', train, dt)
        u = r2 + h
        h = np.maximum(u, 0)
        for lst, v in ((c.t1, t1), (c.xh1, xh1), (c.r1, r1), (c.a1, a1), (c.t2, t2),
                       (c.xh2, xh2), (c.u, u), (c.inv1, inv1), (c.inv2, inv2), (c.masks, m)):
            lst.append(v)
    c.h_out = h
    x = x0
    for l in range(spec.n_cross):
        c.xs.append(x)
        x, s = cross_layer(x, W(f'cross_network.{l}.w.weight')[0], W(f'cross_network.{l}.b'))
        c.ss.append(s)
    c.xL = x
    fin = np.concatenate([h, x], axis=1)            # deep first (train.py:169)
    z = fin @ W('final_linear.weight')[0] + W('final_linear.bias')[0]
    return z, c


def bce_with_logits(z, y):
    """BCEWithLogitsLoss (mean), train.py:206/224; returns (loss, dL/dz)."""
    z = np.asarray(z, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    loss = np.mean(np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z))))
    dz = (1.0 / (1.0 + np.exp(-z)) - y) / z.shape[0]
    return loss, dz


def backward(p, spec: ModelSpec, c: Cache, dz, user, item, cat, dt=np.float64):
    """Autograd backward of forward() (loss.backward(), train.py:225).
    Returns dict name -> grad, embedding grads dense (embedding_dense_backward)."""
    W = lambda k: np.asarray(p[k], dtype=dt)
    g = {}
    dz = np.asarray(dz, dtype=dt)
    H = spec.hidden
    wf = W('final_linear.weight')[0]
    g['final_linear.weight'] = (np.concatenate([c.h_out, c.xL], axis=1).T @ dz)[None, :]
    g['final_linear.bias'] = np.array([dz.sum()], dtype=dt)
    dh = dz[:, None] * wf[:H][None, :]
    dx = dz[:, None] * wf[H:][None, :]
    # cross stack (reverse)
    for l in reversed(range(spec.n_cross)):
        xl, s = c.xs[l], c.ss[l]
        wl = W(f'cross_network.{l}.w.weight')[0]
        g[f'cross_network.{l}.b'] = dx.sum(axis=0)
        gx = (dx * xl).sum(axis=1)
        g[f'cross_network.{l}.w.weight'] = (gx[:, None] * xl).sum(axis=0)[None, :]
        dx = dx * (1.0 + s)[:, None] + gx[:, None] * wl[None, :]
    dx0_cross = dx
    B = c.B

    def bn_back(dr, xh, inv, prefix):
        gam = W(prefix + '.weight')
        g[prefix + '.weight'] = (dr * xh).sum(axis=0)
        g[prefix + '.bias'] = dr.sum(axis=0)
        if c.train:
            return gam * inv / B * (B * dr - dr.sum(axis=0) - xh * (dr * xh).sum(axis=0))
        return dr * gam * inv

    for j in reversed(range(spec.n_res)):
        pre = f'res_blocks.{j}'
        du = dh * (c.u[j] > 0)
        dh_in = du.copy()
        dt2 = bn_back(du, c.xh2[j], c.inv2[j], pre + '.bn2')
        g[pre + '.layer2.weight'] = dt2.T @ c.a1[j]
        g[pre + '.layer2.bias'] = dt2.sum(axis=0)
        da = dt2 @ W(pre + '.layer2.weight')
        if c.masks[j] is not None:
            da = da * c.masks[j]
        dr1 = da * (c.r1[j] > 0)
        dt1 = bn_back(dr1, c.xh1[j], c.inv1[j], pre + '.bn1')
        g[pre + '.layer1.weight'] = dt1.T @ c.h_in[j]
        g[pre + '.layer1.bias'] = dt1.sum(axis=0)
        dh = dh_in + dt1 @ W(pre + '.layer1.weight')
    g['initial_deep_layer.weight'] = dh.T @ c.x0
    g['initial_deep_layer.bias'] = dh.sum(axis=0)
    dx0 = dh @ W('initial_deep_layer.weight') + dx0_cross
    # embedding_dense_backward: scatter-add slices of dx0
    e = spec.emb_dim
    off = 0

    def scatter(name, idx, width):
        nonlocal off
        gt = np.zeros(np.asarray(p[name]).shape, dtype=dt)
        np.add.at(gt, idx, dx0[:, off:off + width])
        off += width
        g[name] = gt

    scatter('user_embedding.weight', user, e)
    scatter('item_embedding.weight', item, e)
    for k, n in enumerate(spec.cat_dims):
        scatter(f'cat_embeddings.{k}.weight', cat[:, k], cat_width(n))
    return g


# --------------------------------------------------------------------------
# bf16 storage emulation of the same step (the precision="bf16" path)
# --------------------------------------------------------------------------
def bf16_round(a) -> np.ndarray:
    """Round to bfloat16 (round-to-nearest-even on the fp32 bits), returned
    as float64 -- the value a bf16 store keeps."""
    f = np.array(a, dtype=np.float32, copy=True, order='C')
    u = f.view(np.uint32)
    r = (u >> 16) & 1
    r += 0x7FFF
    u += r            # wraps only for NaN payloads (not produced here)
    u &= 0xFFFF0000
    return f.astype(np.float64)


def _bf16_as(a, dt):
    f = np.array(a, dtype=np.float32, copy=True, order='C')
    u = f.view(np.uint32)
    r = (u >> 16) & 1
    r += 0x7FFF
    u += r
    u &= 0xFFFF0000
    return f if dt == np.float32 else f.astype(dt)


def train_step_bf16(p: Dict[str, np.ndarray], spec: ModelSpec, user, item, cat, num, y,
                    dropout_masks: Optional[List[np.ndarray]] = None, dt=np.float64):
    """The reference's train step (train.py:155-170 forward, 206/224 BCE, 225
    backward) with every tensor the bf16 path STORES rounded to bf16 at the
    point the kernels store it, the rest in ``dt`` (float64, or float32 for
    full-size runs):

      forward   x0 (GEMM operand), deep weights, h_j, t1_j, a1_j, t2_j, h_{j+1};
                BN statistics of the stored t; cross stack not rounded
      backward  du_j (= dh * [h_{j+1} > 0]), dt2_j, da_j, dt1_j, G = dh_0;
                dW = dY^T X over the stored operands; dx0 = G W0 (fp32 out)

    It isolates kernel errors from bf16's own rounding: the bf16 step's
    gradients are compared to THIS to tight bounds (fp64 vs bf16 storage
    alone differ by ~15 % on the first blocks' weight gradients at cfg3r:
    BN's backward subtracts the batch means of the column gradients,
    amplifying the storage rounding block by block).  Updates the BN running
    statistics in ``p`` as forward() does.  Returns (logits, loss, grads)."""
    R, H, B = spec.n_res, spec.hidden, user.shape[0]
    rb = lambda a: _bf16_as(a, dt)                          # noqa: E731
    W = lambda k: np.asarray(p[k], dtype=dt)               # noqa: E731
    Wb = lambda k: rb(p[k])                                 # noqa: E731
    pdrop = spec.dropout
    inv_keep = dt(np.float32(1.0 / (1.0 - pdrop))) if pdrop > 0 else dt(1.0)
    x0f = gather_x0(p, spec, user, item, cat, num, dt)   # fp32 values, exact
    x0 = rb(x0f)
    h = rb(x0 @ Wb('initial_deep_layer.weight').T + W('initial_deep_layer.bias'))

    def bn_stats(t, prefix):
        mu = t.mean(axis=0, dtype=np.float64)
        var = np.maximum(np.square(t, dtype=np.float64).mean(axis=0) - mu * mu, 0.0)
        rm, rv = p[prefix + '.running_mean'], p[prefix + '.running_var']
        p[prefix + '.running_mean'] = ((1 - BN_MOMENTUM) * rm + BN_MOMENTUM * mu).astype(rm.dtype)
        p[prefix + '.running_var'] = ((1 - BN_MOMENTUM) * rv + BN_MOMENTUM * var * B / (B - 1)).astype(rv.dtype)
        p[prefix + '.num_batches_tracked'] = np.asarray(p[prefix + '.num_batches_tracked']) + 1
        inv = (1.0 / np.sqrt(var + BN_EPS)).astype(np.float32)          # fp32 as the finalize
        sc = np.asarray(p[prefix + '.weight'], np.float32) * inv
        sh = np.asarray(p[prefix + '.bias'], np.float32) - mu.astype(np.float32) * sc
        return mu.astype(np.float32).astype(dt), inv.astype(dt), sc.astype(dt), sh.astype(dt)

    hs, t1s, t2s, a1s, st1, st2 = [h], [], [], [], [], []
    for j in range(R):
        pre = f'res_blocks.{j}'
        t1 = rb(h @ Wb(pre + '.layer1.weight').T + W(pre + '.layer1.bias'))
        s1 = bn_stats(t1, pre + '.bn1')
        a1 = np.maximum(t1 * s1[2] + s1[3], 0)
        if pdrop > 0:
            a1 = a1 * dropout_masks[j].astype(dt) * inv_keep
        a1 = rb(a1)
        t2 = rb(a1 @ Wb(pre + '.layer2.weight').T + W(pre + '.layer2.bias'))
        s2 = bn_stats(t2, pre + '.bn2')
        h = rb(np.maximum(t2 * s2[2] + s2[3] + h, 0))
        t1s.append(t1); t2s.append(t2); a1s.append(a1); st1.append(s1); st2.append(s2)
        hs.append(h)
    x = x0f
    xs, ss = [], []
    for l in range(spec.n_cross):
        xs.append(x)
        x, sl = cross_layer(x, W(f'cross_network.{l}.w.weight')[0], W(f'cross_network.{l}.b'))
        ss.append(sl)
    wf = W('final_linear.weight')[0]
    z = hs[R] @ wf[:H] + x @ wf[H:] + W('final_linear.bias')[0]
    loss, dz = bce_with_logits(z, y)
    dz = dz.astype(dt)

    g = {}
    g['final_linear.weight'] = np.concatenate([hs[R].T @ dz, x.T @ dz])[None, :]
    g['final_linear.bias'] = np.array([dz.sum(dtype=np.float64)])
    dx = dz[:, None] * wf[H:][None, :]
    for l in reversed(range(spec.n_cross)):
        xl, sl = xs[l], ss[l]
        wl = W(f'cross_network.{l}.w.weight')[0]
        g[f'cross_network.{l}.b'] = dx.sum(axis=0)
        gx = (dx * xl).sum(axis=1)
        g[f'cross_network.{l}.w.weight'] = (gx[:, None] * xl).sum(axis=0)[None, :]
        dx = dx * (1.0 + sl)[:, None] + gx[:, None] * wl[None, :]

    def bn_back_b(dr, t, st, prefix):
        mu, inv, _, _ = st
        xh = (t - mu) * inv
        s0, s1 = dr.sum(axis=0, dtype=np.float64), (dr * xh).sum(axis=0, dtype=np.float64)
        g[prefix + '.weight'] = s1
        g[prefix + '.bias'] = s0
        a = np.asarray(p[prefix + '.weight'], np.float32) * inv.astype(np.float32)
        k1 = (a.astype(np.float64) * s1 / B).astype(np.float32)
        k2 = (a.astype(np.float64) * s0 / B).astype(np.float32)
        return rb(a.astype(dt) * dr - k1.astype(dt) * xh - k2.astype(dt))

    dhR = dz[:, None] * wf[:H][None, :]             # gradient wrt h_R (fp32)
    du = rb(dhR * (hs[R] > 0).astype(dt))
    for j in reversed(range(R)):
        pre = f'res_blocks.{j}'
        dt2 = bn_back_b(du, t2s[j], st2[j], pre + '.bn2')
        g[pre + '.layer2.weight'] = dt2.T @ a1s[j]
        g[pre + '.layer2.bias'] = np.zeros(H, dt)    # exactly 0 (BN removes it)
        da = dt2 @ Wb(pre + '.layer2.weight') * inv_keep
        da = rb(da) * (a1s[j] != 0).astype(dt)
        dt1 = bn_back_b(da, t1s[j], st1[j], pre + '.bn1')
        g[pre + '.layer1.weight'] = dt1.T @ hs[j]
        g[pre + '.layer1.bias'] = np.zeros(H, dt)
        G = rb(dt1 @ Wb(pre + '.layer1.weight') + du)
        du = G * (hs[j] > 0).astype(dt) if j > 0 else G
    G = du
    g['initial_deep_layer.weight'] = G.T @ x0
    g['initial_deep_layer.bias'] = G.sum(axis=0, dtype=np.float64)
    dx0 = G @ Wb('initial_deep_layer.weight') + dx
    e = spec.emb_dim
    off = 0

    def scatter(name, idx, width):
        nonlocal off
        gt = np.zeros(np.asarray(p[name]).shape, dtype=dt)
        np.add.at(gt, idx, dx0[:, off:off + width])
        off += width
        g[name] = gt

    scatter('user_embedding.weight', user, e)
    scatter('item_embedding.weight', item, e)
    for k, n in enumerate(spec.cat_dims):
        scatter(f'cat_embeddings.{k}.weight', cat[:, k], cat_width(n))
    return z, loss, g


# --------------------------------------------------------------------------
# optimizer (train.py:201-204, 226)
# --------------------------------------------------------------------------
def adam_step(param, grad, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8,
              weight_decay=0.0, decoupled=True):
    """One torch.optim.AdamW (decoupled=True) / Adam (decoupled=False) step,
    single-tensor algorithm; returns new (param, m, v).  ``step`` is the
    1-based step count after increment."""
    param = param.astype(np.float64)
    grad = grad.astype(np.float64)
    if decoupled:
        param = param * (1 - lr * weight_decay)
    elif weight_decay != 0:
        grad = grad + weight_decay * param
    m = beta1 * m + (1 - beta1) * grad
    v = beta2 * v + (1 - beta2) * grad * grad
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = np.sqrt(v) / math.sqrt(bc2) + eps
    param = param - (lr / bc1) * m / denom
    return param, m, v


# --------------------------------------------------------------------------
# candidate generation: cosine kNN (main.py:268-270, 196-203, 299-302)
# --------------------------------------------------------------------------
def cosine_kneighbors(table: np.ndarray, queries: np.ndarray, k: int):
    """sklearn NearestNeighbors(metric='cosine', algorithm='brute').kneighbors
    restated: normalise rows, dist = clip(1 - q.x, 0, 2) (fp32), then
    argpartition(k-1) + argsort.  Ties are ordered by index here (stable),
    where sklearn's argsort is unstable; tests compare modulo ties."""
    t = np.asarray(table, dtype=np.float32)
    q = np.asarray(queries, dtype=np.float32)

    def normalize(a):
        n = np.sqrt(np.einsum('ij,ij->i', a, a))
        n[n == 0.0] = 1.0
        return a / n[:, None]

    s = normalize(q) @ normalize(t).T
    d = np.clip(1.0 - s, 0.0, 2.0).astype(np.float32)
    idx = np.argsort(d, axis=1, kind='stable')[:, :k]
    return np.take_along_axis(d, idx, axis=1), idx


# --------------------------------------------------------------------------
# serving: candidate union, ranking order, MMR (main.py:196-203, 325, 133-169)
# --------------------------------------------------------------------------
def candidate_union(positive_rows, knn_idx):
    """_generate_candidates' set (main.py:196-203): the positives plus each
    one's neighbours with position 0 dropped (main.py:201), as ascending rows."""
    s = set(int(r) for r in positive_rows)
    for row in np.asarray(knn_idx):
        s.update(int(r) for r in row[1:] if r >= 0)
    return np.asarray(sorted(s), dtype=np.int64)


def rank_by_score(scores):
    """sorted(zip(scores, ids), key=score, reverse=True) (main.py:325): a
    stable descending order (equal scores keep their input order)."""
    return np.argsort(-np.asarray(scores, dtype=np.float32), kind='stable')


def mmr_rerank(emb, rows, scores, lam, top_k=20):
    """rerank_with_mmr (main.py:133-169) on embedding rows (-1 = id absent from
    item_id_mapping) in ranked order; returns positions into the ranked list.
    cosine_similarity as sklearn: normalize (zero rows stay zero), then dot."""
    emb = np.asarray(emb, dtype=np.float32)
    n = len(rows)
    if n == 0:
        return []

    def unit(v):
        nv = np.sqrt(np.dot(v, v))
        return v / nv if nv > 0 else v

    final = [0]
    remaining = list(range(1, n))
    while len(final) < min(top_k, n):
        best, best_score = -1, -np.inf
        sel = [rows[p] for p in final if rows[p] >= 0]
        for p in remaining:
            if rows[p] < 0:
                continue
            if not sel:
                ms = np.float32(0.0)
            else:
                c = unit(emb[rows[p]])
                ms = max(np.float32(np.dot(c, unit(emb[s]))) for s in sel)
            m = np.float32(lam) * np.float32(scores[p]) - np.float32(1 - lam) * ms
            if m > best_score:
                best, best_score = p, m
        if best == -1:
            break
        final.append(best)
        remaining.remove(best)
    return final
