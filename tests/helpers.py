"""Shared test helpers (build our model from a golden recipe, compare, ...)."""
from __future__ import annotations

import numpy as np
import torch

import golden_common as gc
import dcnr_oracle as orc


def our_model(cfg, precision="fp32", seed=gc.WEIGHT_SEED):
    import dcnr
    torch.manual_seed(seed)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), precision=precision)
    gc.perturb_state(m, seed + 1)
    return m


def check_checksums(model, fx):
    ck = gc.state_checksums(model)
    names = list(fx["ck_names"])
    assert names == list(ck.keys()), "state_dict keys differ from the reference"
    got = np.stack([ck[k] for k in names])
    np.testing.assert_allclose(got, fx["ck"], rtol=1e-12, atol=1e-9)


def np_state(model):
    return {k: v.detach().cpu().double().numpy().copy() for k, v in model.state_dict().items()}


def spec_of(cfg, dropout=None):
    p = dict(cfg["params"])
    if dropout is not None:
        p["dropout"] = dropout
    return orc.spec_from_params(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"], p)


def to_dev(dev, *arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in arrs]


def logits_err(z, ref):
    """Element-wise |dz| / max(|ref|, 1) (SURVEY 8c criterion)."""
    z = np.asarray(z, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(z - ref) / np.maximum(np.abs(ref), 1.0)))


def grad_rel(g, ref):
    ref = np.asarray(ref, np.float64)
    g = np.asarray(g, np.float64)
    return float(np.linalg.norm(g - ref) / max(np.linalg.norm(ref), 1e-30))


def assert_grads_close(grads: dict, ref: dict, rtol=5e-3, atol=1e-7, names=None):
    bad = []
    for k in (names or ref.keys()):
        g, r = grads[k], ref[k]
        if np.abs(g - r).max() <= atol:
            continue
        e = grad_rel(g, r)
        if e > rtol:
            bad.append((k, e, float(np.abs(g - r).max())))
    assert not bad, f"grad mismatches: {bad}"


def dropout_mask_np(seed: int, layer: int, B: int, H: int, p: float) -> np.ndarray:
    """Host replica of libdcnr's counter-based dropout keep-test
    (csrc/dcnr_internal.h dropout_keep): keep(seed, layer, row, col)."""
    M = np.uint64
    with np.errstate(over="ignore"):
        x = M(seed) ^ (M(0x9E3779B97F4A7C15) * M(layer + 1))
        rows = np.arange(B, dtype=np.uint64)[:, None]
        cols = np.arange(H, dtype=np.uint64)[None, :]
        x = x + rows * M(0x100000001B3) + cols * M(0xC2B2AE3D27D4EB4F)
        x = x ^ (x >> M(30)); x = x * M(0xBF58476D1CE4E5B9)
        x = x ^ (x >> M(27)); x = x * M(0x94D049BB133111EB)
        x = x ^ (x >> M(31))
    thresh = np.uint64(min(4294967295.0, float(np.float32(p)) * 4294967296.0))
    return ((x >> M(32)) >= thresh).astype(np.float64)
