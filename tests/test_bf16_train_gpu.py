"""End-to-end parity of the BENCHMARKED training path: bf16 deep tower
(gemm_ws BN-statistics forward epilogues, the DROP_BN / RESID_BN dX
epilogues with 1-bit keep masks, gemm_dw weight gradients), dropout 0.6,
train-mode BatchNorm, BCE, backward (train.py:112-122, 155-170, 206, 225).

Why these bounds.  The reference computes in fp32; the bf16 path STORES
activations and gradients in bf16 (2^-9 relative rounding per store).  At
these model states the gradient is very sensitive to such perturbations:
1e-6 relative noise on the weights alone moves the deep tower's weight
gradients by 1.5e-3 in fp64 (measured with the oracle), 1e-4 by 4 %.  bf16
storage alone -- the oracle's ``train_step_bf16``, which rounds exactly the
tensors the kernels store -- is 10-16 % away from fp64 on the first blocks'
weight gradients, and a float32-arithmetic run of that same emulation is
8 % away from its float64 run.  So no bf16 implementation can be pinned to
another element-wise end to end; the kernels are pinned STAGE BY STAGE
(each stored tensor recomputed from the kernel's own stored inputs,
tests/test_stages_gpu.py).  End to end, per tensor:

  cos(g, g_ref) >= COS_MIN and ||g - g_ref||/||g_ref|| <= REL_MAX
  ||g - g64|| / ||g64|| <= EMU_FACTOR * ||g_emu - g64|| / ||g64|| + 2e-3
      (the kernels' distance from fp64 is that of bf16 storage itself)
  logits ||dz||/||z|| <= 1e-2; running statistics <= 1e-2; num_batches exact

A sign, transpose, mask-bit or wrong-operand error in any epilogue fails the
cosine floor.  The pre-BN Linear biases have an exactly-zero gradient in the
bf16 path (BN removes them) and are checked absolutely.
"""
import numpy as np
import pytest
import torch

import dcnr_oracle as orc
import golden_common as gc
from conftest import golden
from helpers import dropout_mask_np, grad_rel, np_state, our_model, spec_of, to_dev

pytestmark = pytest.mark.gpu

COS_MIN = 0.98
REL_MAX = 0.25
EMU_FACTOR = 1.5
LOGIT_TOL = 1e-2
BN_TOL = 1e-2


def _train_step(model, dev, seed, u, i, c, n, y):
    import dcnr
    torch.manual_seed(seed)
    model.train()
    model.zero_grad(set_to_none=True)
    z = model(u, i, c, n)
    loss = dcnr.BCEWithLogitsLoss()(z, y)
    loss.backward()
    torch.cuda.synchronize()
    return z.detach(), float(loss.detach())


def _pre_bn_bias(k):
    return ".layer" in k and k.endswith(".bias")


def _cos(a, b):
    a, b = np.ravel(a), np.ravel(b)
    return float(a @ b / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-300))


def _check(model, ref, label, to_np, emu=None, ref64=None):
    """Per-tensor cosine / relative-error bounds (module docstring); with
    ``emu`` (bf16-storage emulation) and ``ref64`` the kernels' distance from
    fp64 is also bounded by the emulation's."""
    print(f"\n  {label}: tensor, cos, ||dg||/||g||" + (", emulation's" if emu else ""))
    bad = []
    for k, p in model.named_parameters():
        g = to_np(p.grad.detach())
        r = to_np(ref[k])
        if _pre_bn_bias(k):
            assert np.abs(g).max() == 0.0, k
            continue
        c, e = _cos(g, r), grad_rel(g, r)
        line = f"    {k:40s} {c:.5f} {e:.3e}"
        ok = c >= COS_MIN and e <= REL_MAX
        if emu is not None:
            ee = grad_rel(to_np(emu[k]), r)
            line += f" {ee:.3e}"
            ok = ok and e <= EMU_FACTOR * ee + 2e-3
        print(line)
        if not ok:
            bad.append(k)
    assert not bad, bad


def test_bf16_train_step_cfg3r_dropout(dev):
    """cfg3r (D=456, H=512, 4 res, 3 cross), B=1024, p=0.6: every gradient,
    logits, loss and BN running statistics of the bf16 step against the fp64
    oracle fed the same dropout masks, and the kernels' distance from fp64
    against bf16 storage's own (oracle train_step_bf16)."""
    import copy
    from dcnr.model import dropout_seed
    fx = golden("f3_cfg3r_train.npz")
    cfg = dict(gc.CFG3R, params=dict(gc.CFG3R["params"], dropout=0.6))
    spec = spec_of(cfg)
    m = our_model(cfg, precision="bf16").to(dev)
    sd = np_state(m)
    sde = copy.deepcopy(sd)
    u, i, c, n, y = fx["user"], fx["item"], fx["cat"], fx["num"], fx["y"]
    B = u.shape[0]
    torch.manual_seed(99)
    seed = dropout_seed(dev, advance=False)          # what the forward will draw
    z, loss = _train_step(m, dev, 99, *to_dev(dev, u, i, c, n, y))
    masks = [dropout_mask_np(seed, j, B, spec.hidden, 0.6) for j in range(spec.n_res)]
    zr, cache = orc.forward(sd, spec, u, i, c, n, train=True, dropout_masks=masks)
    lr, dz = orc.bce_with_logits(zr, y)
    gr = orc.backward(sd, spec, cache, dz, u, i, c)
    _, _, ge = orc.train_step_bf16(sde, spec, u, i, c, n, y, masks)
    z = z.cpu().double().numpy()
    assert np.linalg.norm(z - zr) / np.linalg.norm(zr) <= LOGIT_TOL
    assert abs(loss - lr) <= 5e-3
    _check(m, gr, "bf16 kernels vs fp64 oracle",
           lambda t: np.asarray(t.cpu().double().numpy() if torch.is_tensor(t) else t, np.float64),
           emu=ge, ref64=gr)
    sd_after = np_state(m)
    for k in sd:
        if "running" in k:
            e = np.linalg.norm(sd_after[k] - sd[k]) / max(np.linalg.norm(sd[k]), 1e-12)
            assert e <= BN_TOL, (k, e)
        if "num_batches_tracked" in k:
            assert int(sd_after[k]) == int(sd[k]) == 1, k


def test_bf16_train_step_vs_fp32_full_size(dev):
    """configs[2] at B=131072, p=0.6 (the bench's step): the bf16 step vs the
    fp32 step (f32 MFMA + rowwise kernels, pinned element-wise to the
    reference's fixtures) on the same weights, inputs and dropout seed --
    every gradient, logits, running statistics, num_batches_tracked."""
    import copy
    import dcnr
    cfg = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
               n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3,
                                    n_res_blocks=4, dropout=0.6))
    torch.manual_seed(7)
    m32 = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                          dict(cfg["params"]), precision="fp32")
    gc.perturb_state(m32, 8)
    m16 = copy.deepcopy(m32)
    m16.precision = "bf16"
    m32, m16 = m32.to(dev), m16.to(dev)
    B = 131072
    g = torch.Generator(device=dev).manual_seed(3)
    u = torch.randint(0, cfg["n_users"], (B,), device=dev, generator=g)
    i = torch.randint(0, cfg["n_items"], (B,), device=dev, generator=g)
    c = torch.randint(0, 1000, (B, 12), device=dev, generator=g)
    n = torch.rand((B, 8), device=dev, generator=g)
    y = (torch.rand((B,), device=dev, generator=g) < 0.5).float()
    z32, l32 = _train_step(m32, dev, 11, u, i, c, n, y)
    z16, l16 = _train_step(m16, dev, 11, u, i, c, n, y)
    assert ((z16 - z32).norm() / z32.norm()).item() <= LOGIT_TOL
    assert abs(l16 - l32) <= 5e-3
    p32 = {k: p.grad for k, p in m32.named_parameters()}
    _check(m16, p32, "bf16 vs fp32 kernels, B=131072", lambda t: t.double().cpu().numpy())
    s32 = m32.state_dict()
    for k, v in m16.state_dict().items():
        if "running" in k:
            e = ((v.double() - s32[k].double()).norm() / s32[k].double().norm()).item()
            assert e <= BN_TOL, (k, e)
        if "num_batches_tracked" in k:
            assert int(v) == int(s32[k]) == 1, k
