"""Shared recipes for the golden fixtures (used by make_golden.py, which runs
the reference, and by the tests, which run our build + the oracle).

Weights are NOT stored in the fixtures: they are regenerated from a torch
seed by constructing the model (the reference's ``DCN_RecSys`` and ours
consume the torch RNG identically -- same submodules in the same order,
train.py:136-153), then perturbed by ``perturb_state`` so that BN statistics,
BN affine parameters and cross-layer biases are non-trivial.  Each fixture
stores per-tensor checksums of the weights so a mismatch in regeneration is
detected before any numeric comparison.
"""
from __future__ import annotations

import numpy as np
import torch

CFG1 = dict(n_users=10_000, n_items=5_000, cat_dims={f"c{i}": 250 for i in range(8)}, n_num=4,
            params=dict(emb_dim=16, hidden_dim=128, n_cross_layers=2, n_res_blocks=2, dropout=0.0))
# reduced cfg3 shape: D=456, H=512, 4 res, 3 cross
CFG3R = dict(n_users=4096, n_items=1024, cat_dims={f"c{i}": 1000 for i in range(12)}, n_num=8,
             params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4, dropout=0.0))
# odd shapes: non-multiple-of-8 widths, single cat table of width 2, H not a multiple of 64
CFG_ODD = dict(n_users=37, n_items=11, cat_dims={"a": 3, "b": 17, "c": 1}, n_num=3,
               params=dict(emb_dim=24, hidden_dim=96, n_cross_layers=4, n_res_blocks=3, dropout=0.0))

WEIGHT_SEED = 42


def build(cls, cfg, seed=WEIGHT_SEED):
    torch.manual_seed(seed)
    m = cls(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"], dict(cfg["params"]))
    perturb_state(m, seed + 1)
    return m


@torch.no_grad()
def perturb_state(model, seed):
    """Make BN stats/affine and cross biases non-trivial, deterministically."""
    g = torch.Generator().manual_seed(seed)
    sd = model.state_dict()
    for k in sorted(sd.keys()):
        t = sd[k]
        if k.endswith("running_mean"):
            t.copy_(torch.randn(t.shape, generator=g) * 0.1)
        elif k.endswith("running_var"):
            t.copy_(torch.rand(t.shape, generator=g) + 0.5)
        elif ".bn" in k and k.endswith(".weight"):
            t.copy_(torch.rand(t.shape, generator=g) + 0.5)
        elif ".bn" in k and k.endswith(".bias"):
            t.copy_(torch.randn(t.shape, generator=g) * 0.1)
        elif k.startswith("cross_network") and k.endswith(".b"):
            t.copy_(torch.randn(t.shape, generator=g) * 0.05)


def make_inputs(cfg, B, seed):
    rng = np.random.default_rng(seed)
    user = rng.integers(0, cfg["n_users"], size=B, dtype=np.int64)
    item = rng.integers(0, cfg["n_items"], size=B, dtype=np.int64)
    cards = list(cfg["cat_dims"].values())
    cat = np.stack([rng.integers(0, c, size=B, dtype=np.int64) for c in cards], axis=1) \
        if cards else np.zeros((B, 0), np.int64)
    num = rng.random((B, cfg["n_num"]), dtype=np.float32)
    y = (rng.random(B) < 0.5).astype(np.float32)
    return user, item, cat, num, y


def state_checksums(model):
    out = {}
    for k, v in model.state_dict().items():
        a = v.detach().double().cpu().numpy()
        out[k] = np.array([a.sum(), np.abs(a).sum()], dtype=np.float64)
    return out


def knn_table(seed=7, n=20_000, d=64, n_dup=64):
    """Item-embedding table with planted duplicate (and scaled-duplicate)
    rows, so ties / exact-zero distances are exercised."""
    rng = np.random.default_rng(seed)
    t = rng.standard_normal((n, d)).astype(np.float32)
    src = rng.choice(n, size=n_dup, replace=False)
    dst = rng.choice(np.setdiff1d(np.arange(n), src), size=n_dup, replace=False)
    t[dst[: n_dup // 2]] = t[src[: n_dup // 2]]                    # exact duplicates
    t[dst[n_dup // 2:]] = 3.0 * t[src[n_dup // 2:]]                # same direction
    q_rows = np.concatenate([src[:8], rng.choice(n, size=8, replace=False)])
    return t, q_rows
