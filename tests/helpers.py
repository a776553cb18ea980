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


def _fmix32(x):
    U = np.uint32
    x = x ^ (x >> U(16)); x = x * U(0x85EBCA6B)
    x = x ^ (x >> U(13)); x = x * U(0xC2B2AE35)
    return x ^ (x >> U(16))


def dropout_mask_np(seed: int, layer: int, B: int, H: int, p: float) -> np.ndarray:
    """Host replica of libdcnr's counter-based dropout mask
    (csrc/dcnr_internal.h dropout_bits): 32 bits per (row, column pair), low
    16 bits for the even column, high 16 for the odd one; keep iff the 16
    bits >= round(p * 65536)."""
    U = np.uint32
    with np.errstate(over="ignore"):
        rows = np.arange(B, dtype=np.uint64).astype(U)[:, None]
        pairs = (np.arange(H, dtype=np.uint32) >> U(1))[None, :]
        x = _fmix32(rows * U(0x9E3779B1) ^ U(seed & 0xFFFFFFFF) ^ U((layer * 0x7FEB352D) & 0xFFFFFFFF))
        x = _fmix32((x + pairs * U(0x846CA68B)) ^ U(seed >> 32))
    odd = (np.arange(H) & 1).astype(bool)[None, :]
    bits16 = np.where(odd, x >> U(16), x & U(0xFFFF))
    thresh = min(65536, int(np.floor(float(np.float32(p)) * 65536.0 + 0.5)))
    return (bits16.astype(np.int64) >= thresh).astype(np.float64)


def dropout_mask_torch(seed: int, layer: int, B: int, H: int, p: float, device) -> "torch.Tensor":
    """dropout_mask_np on the device (int64 arithmetic kept to 32 bits): the
    same keep mask, for full-size batches."""
    M = 0xFFFFFFFF

    def fmix(x):
        x = x ^ (x >> 16)
        x = (x * 0x85EBCA6B) & M
        x = x ^ (x >> 13)
        x = (x * 0xC2B2AE35) & M
        return x ^ (x >> 16)

    rows = torch.arange(B, dtype=torch.int64, device=device)[:, None]
    pairs = (torch.arange(H, dtype=torch.int64, device=device) >> 1)[None, :]
    x = fmix(((rows * 0x9E3779B1) & M) ^ (seed & M) ^ ((layer * 0x7FEB352D) & M))
    x = fmix((((x + pairs * 0x846CA68B) & M) ^ ((seed >> 32) & M)))
    odd = (torch.arange(H, device=device) & 1).bool()[None, :]
    bits16 = torch.where(odd, x >> 16, x & 0xFFFF)
    thresh = min(65536, int(np.floor(float(np.float32(p)) * 65536.0 + 0.5)))
    return (bits16 >= thresh)
