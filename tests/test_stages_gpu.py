"""Stage-by-stage parity of the bf16 training step (the benchmarked path).

End to end a bf16 step cannot be pinned element-wise to any other
implementation (tests/test_bf16_train_gpu.py explains the sensitivity), but
every STAGE can: each tensor the kernels store is recomputed here, in torch
fp32/fp64 on the device, from the kernels' OWN stored inputs of that stage,
and compared.  The workspace keeps every block's backward buffers
(DCNR_FLAG_KEEP_INTERMEDIATES) and tells where each tensor lives
(dcnr_workspace_offset).  Stages and reference lines:

  forward  (train.py:155-170, ResBlock 112-122)
    x0          gather + concat, bf16 store                       exact
    h0, t1, t2  Linear (bf16 operands, fp32 accumulate) + bias     <= BF16_ULPS ulp
    BN stats    mean / invstd of the stored t (fp64 sums)          rel 1e-5
    a1          dropout(relu(t1 * scale + shift)), keep mask       <= BF16_ULPS ulp
    h_{j+1}     relu(t2 * scale + shift + h_j)                     <= BF16_ULPS ulp
    masks       1-bit [a1 != 0], [h_j > 0] images                  exact
    logits      h_R . w_f[:H] + zc + b_f                           rel 1e-5
    sc          s_l, x_0 . w_m, x_0 . w_f[H:] (cross scalars)      rel 1e-5
  backward (loss.backward(), train.py:225)
    du_{R-1}    dz w_f[:H] * [h_R > 0]                             <= BF16_ULPS ulp
    dt2, dt1    BN backward apply (coefficients from fp64 sums)     <= BF16_ULPS ulp
    da          (dt2 W2) / (1-p) * [a1 != 0]                        <= BF16_ULPS ulp
    du_{j-1}    (dt1 W1 + du_j) * [h_j > 0];  G = dt1_0 W1 + du_0  <= BF16_ULPS ulp
    dW, db, dgamma, dbeta, dW_f, cross, embedding grads (fp32 sums)  rel 2e-4
    dx0_cross   sum_k xcoef_k V_k (low-rank cross backward)         rel 2e-4
    (the cross weight grads' x_0 part is summed over the stored bf16 x0)

A bf16 value within BF16_ULPS units in the last place (plus ACC_EPS times
the magnitude of the summed terms): the kernels and this recomputation
accumulate in different orders, which moves a value across a bf16 rounding
boundary now and then (the fraction of such elements is printed and bounded
by FLIP_FRAC).
"""
import numpy as np
import pytest
import torch

import golden_common as gc
from helpers import dropout_mask_torch

pytestmark = pytest.mark.gpu

BF16_ULPS = 1
ACC_EPS = 2.0 ** -18     # fp32 accumulation-order allowance, relative to the summed |terms|
FLIP_FRAC = 0.02
REL = 2e-4


def _cfg(full):
    if full == "h384":   # K = 384 < 512: the fused BN-backward operand's partial last chunks
        return dict(n_users=50_000, n_items=5_000, cat_dims={f"c{k}": 100 for k in range(4)},
                    n_num=8, params=dict(emb_dim=32, hidden_dim=384, n_cross_layers=2,
                                         n_res_blocks=3, dropout=0.6)), 8192
    if full:
        return dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
                    n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3,
                                         n_res_blocks=4, dropout=0.6)), 131072
    return dict(gc.CFG3R, params=dict(gc.CFG3R["params"], dropout=0.6)), 1024


def bf(t):
    return t.to(torch.bfloat16).float()


def ulp_bf16(x):
    """One bf16 unit in the last place at |x| (8 significant bits)."""
    a = x.abs().clamp_min(1e-30)
    return torch.exp2(torch.floor(torch.log2(a)) - 7)


def check_bf16(name, got, ref, stats, scale):
    """``scale``: the magnitude of the terms that were summed into each value
    (|X| @ |W|^T for a GEMM, the sum of |terms| for an elementwise stage):
    different fp32 summation orders / FMA contractions differ by a few fp32
    ulps of it, which near a cancellation can exceed a bf16 ulp of the
    result."""
    got, ref = got.float(), ref.float()
    d = (got - ref).abs()
    assert torch.isfinite(got).all(), name
    tol = BF16_ULPS * ulp_bf16(ref) + ACC_EPS * scale.float() + 1e-30
    bad = d > tol * 1.0001
    # values that are exactly zero on one side only: legitimate only as a
    # rounding flip of a tiny value (never for masked elements)
    nb = int(bad.sum())
    flips = float((got != bf(ref)).float().mean())   # vs the reference rounded to bf16
    stats.append((name, flips, float(d.max())))
    assert nb == 0, (name, nb, float(d.max()), got[bad][:5].tolist(), ref[bad][:5].tolist())
    assert flips <= FLIP_FRAC, (name, flips)


def check_rel(name, got, ref, tol=REL):
    got, ref = got.double(), ref.double()
    e = ((got - ref).norm() / ref.norm().clamp_min(1e-300)).item()
    assert e <= tol, (name, e)


def unpack_bits(b, B, Hp):
    sh = torch.arange(8, device=b.device, dtype=torch.uint8)
    return ((b.view(B, Hp // 8)[:, :, None] >> sh) & 1).reshape(B, Hp).bool()


@pytest.mark.parametrize("full", [False, True, "h384"], ids=["cfg3r_B1024", "cfg2_B131072", "h384_B8192"])
def test_bf16_step_stage_by_stage(dev, full):
    import dcnr
    from dcnr import _lib
    from dcnr.model import dropout_seed, run_backward, run_forward
    from dcnr.ops import bce_with_logits
    cfg, B = _cfg(full)
    torch.manual_seed(7)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), precision="bf16")
    gc.perturb_state(m, 8)
    m = m.to(dev).train()
    m.keep_intermediates = True
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator(device=dev).manual_seed(5)
    K = len(cfg["cat_dims"])
    cards = list(cfg["cat_dims"].values())
    u = torch.randint(0, cfg["n_users"], (B,), device=dev, generator=g)
    i = torch.randint(0, cfg["n_items"], (B,), device=dev, generator=g)
    c = torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in cards], 1)
    n = torch.rand((B, cfg["n_num"]), device=dev, generator=g)
    y = (torch.rand((B,), device=dev, generator=g) < 0.5).float()
    p = cfg["params"]["dropout"]
    R, H = cfg["params"]["n_res_blocks"], cfg["params"]["hidden_dim"]
    Hp = (H + 7) // 8 * 8
    D = m._dims["input_dim"]
    Dp = (D + 7) // 8 * 8

    seed = dropout_seed(dev)
    logits, ws = run_forward(m, True, seed, u, i, c, n)
    loss, dz = bce_with_logits(logits, y)
    params = m.param_tensors()
    grads = [torch.empty_like(q) for q in params]
    run_backward(m, u, i, c, n, dz, ws, grads, seed)
    torch.cuda.synchronize()
    gd = dict(zip([k for k, _ in m.named_parameters()], grads))

    def T(kind, idx=0, cols=Hp, dtype=torch.bfloat16, rows=B):
        off = m.workspace_offset(B, _lib.TRAIN, kind, idx)
        assert off >= 0, (kind, idx)
        nb = rows * cols * torch.tensor([], dtype=dtype).element_size()
        return ws[off:off + nb].view(dtype).view(rows, cols)

    def V(kind, idx):   # fp32 [Hp] vector
        return T(kind, idx, cols=Hp, dtype=torch.float32, rows=1)[0]

    def bits(kind, idx):
        off = m.workspace_offset(B, _lib.TRAIN, kind, idx)
        assert off >= 0, (kind, idx)
        return unpack_bits(ws[off:off + B * Hp // 8], B, Hp)

    f32 = torch.float32
    Wb = lambda k: bf(sd0[k].float())                # noqa: E731 (bf16-packed weights)
    pad = lambda w, r, cl: torch.nn.functional.pad(w, (0, cl - w.shape[1], 0, r - w.shape[0]))  # noqa: E731
    stats = []

    # ---- forward -------------------------------------------------------
    parts = [sd0["user_embedding.weight"][u], sd0["item_embedding.weight"][i]]
    parts += [sd0[f"cat_embeddings.{k}.weight"][c[:, k]] for k in range(K)]
    x0f = torch.cat(parts + [n], 1)
    x0 = T("x0", cols=Dp).float()[:, :D]
    assert torch.equal(x0, bf(x0f)), "x0 gather"
    W0 = Wb("initial_deep_layer.weight")
    h = T("h", 0).float()
    check_bf16("h0", h[:, :H], x0 @ W0.T + sd0["initial_deep_layer.bias"], stats,
               x0.abs() @ W0.abs().T + sd0["initial_deep_layer.bias"].abs())
    keep = [dropout_mask_torch(seed, j, B, H, p, dev) for j in range(R)]
    inv_keep = float(np.float32(1.0 / (1.0 - p)))
    hs = [h]
    for j in range(R):
        pre = f"res_blocks.{j}"
        for l, (tk, bi) in enumerate((("t1", 2 * j), ("t2", 2 * j + 1))):
            Xin = hs[j] if l == 0 else a1
            t = T(tk, j).float()
            W = pad(Wb(f"{pre}.layer{l + 1}.weight"), Hp, Hp)
            b = pad(sd0[f"{pre}.layer{l + 1}.bias"][None], 1, Hp)[0]
            check_bf16(f"{tk}[{j}]", t[:, :H], (Xin @ W.T + b)[:, :H], stats,
                       (Xin.abs() @ W.abs().T + b.abs())[:, :H])
            t64 = t[:, :H].double()
            mu = t64.mean(0)
            var = (t64 * t64).mean(0) - mu * mu
            check_rel(f"mean{bi}", V("bn_mean", bi)[:H], mu, 1e-5)
            check_rel(f"invstd{bi}", V("bn_invstd", bi)[:H], 1.0 / torch.sqrt(var + 1e-5), 1e-5)
            gam = sd0[f"{pre}.bn{l + 1}.weight"].float()
            check_rel(f"scale{bi}", V("bn_scale", bi)[:H], gam * V("bn_invstd", bi)[:H], 1e-6)
            sc, sh = V("bn_scale", bi), V("bn_shift", bi)
            if l == 0:
                a1 = T("a1", j).float()
                ref = torch.clamp_min(t * sc + sh, 0)[:, :H] * keep[j].float() * inv_keep
                check_bf16(f"a1[{j}]", a1[:, :H], ref, stats,
                           ((t * sc).abs() + sh.abs())[:, :H] * inv_keep)
                assert torch.equal(bits("mask_a1", j)[:, :H], a1[:, :H] != 0), f"mask_a1[{j}]"
            else:
                hn = T("h", j + 1).float()
                check_bf16(f"h[{j + 1}]", hn[:, :H], torch.clamp_min(t * sc + sh + hs[j], 0)[:, :H],
                           stats, ((t * sc).abs() + sh.abs() + hs[j].abs())[:, :H])
                if j + 1 < R:
                    assert torch.equal(bits("mask_h", j + 1)[:, :H], hn[:, :H] > 0), f"mask_h[{j + 1}]"
                hs.append(hn)
    wf = sd0["final_linear.weight"][0].float()
    zc = T("zc", cols=1, dtype=f32)[:, 0]
    check_rel("logits", logits, hs[R][:, :H] @ wf[:H] + zc + sd0["final_linear.bias"][0], 1e-5)
    # cross network in fp64 from the fp32 gathered rows: zc = x_L . w_f[H:]
    x = x0f.double()
    xs, ss = [], []
    for l in range(cfg["params"]["n_cross_layers"]):
        xs.append(x)
        wl = sd0[f"cross_network.{l}.w.weight"][0].double()
        s_ = x @ wl
        ss.append(s_)
        x = x + x * s_[:, None] + sd0[f"cross_network.{l}.b"].double()
    check_rel("zc", zc, x @ wf[H:].double(), 1e-5)
    # the cross backward's saved scalars: s_l, u_m = x_0 . w_m, u_f = x_0 . w_f[H:]
    Lc = cfg["params"]["n_cross_layers"]
    scs = T("sc", cols=2 * Lc + 1, dtype=f32)
    us = [x0f.double() @ sd0[f"cross_network.{m}.w.weight"][0].double() for m in range(Lc)]
    for l in range(Lc):
        check_rel(f"s[{l}]", scs[:, l], ss[l], 1e-5)
        check_rel(f"u[{l}]", scs[:, Lc + l], us[l], 1e-5)
    check_rel("u_f", scs[:, 2 * Lc], x0f.double() @ wf[H:].double(), 1e-5)

    # ---- backward ------------------------------------------------------
    def bn_back(dr, t, bi, gam_key):
        mu, inv = V("bn_mean", bi)[:H], V("bn_invstd", bi)[:H]
        xh = (t[:, :H] - mu) * inv
        s0 = dr[:, :H].double().sum(0)
        s1 = (dr[:, :H].double() * xh.double()).sum(0)
        a = sd0[gam_key].float() * inv
        k1 = (a.double() * s1 / B).float()
        k2 = (a.double() * s0 / B).float()
        return a * dr[:, :H] - k1 * xh - k2, s0, s1, (a * dr[:, :H]).abs() + (k1 * xh).abs() + k2.abs()

    du = T("du", R - 1).float()
    ref = dz[:, None] * wf[:H] * (hs[R][:, :H] > 0).float()
    check_bf16(f"du[{R - 1}]", du[:, :H], ref, stats, ref.abs())
    check_rel("dW_f[:H]", gd["final_linear.weight"][0, :H], hs[R][:, :H].double().T @ dz.double())
    for j in reversed(range(R)):
        pre = f"res_blocks.{j}"
        du = T("du", j).float()
        dt2 = T("dt2", j).float()
        ref, s0, s1, sc_ = bn_back(du, T("t2", j).float(), 2 * j + 1, f"{pre}.bn2.weight")
        check_bf16(f"dt2[{j}]", dt2[:, :H], ref, stats, sc_)
        check_rel(f"dbeta2[{j}]", gd[f"{pre}.bn2.bias"], s0)
        check_rel(f"dgamma2[{j}]", gd[f"{pre}.bn2.weight"], s1)
        a1 = T("a1", j).float()
        check_rel(f"dW2[{j}]", gd[f"{pre}.layer2.weight"], dt2[:, :H].double().T @ a1[:, :H].double())
        assert gd[f"{pre}.layer2.bias"].abs().max() == 0
        W2 = pad(Wb(f"{pre}.layer2.weight"), Hp, Hp)
        da = T("da", j).float()
        check_bf16(f"da[{j}]", da[:, :H], ((dt2 @ W2) * inv_keep * (a1 != 0).float())[:, :H], stats,
                   ((dt2.abs() @ W2.abs()) * inv_keep)[:, :H])
        dt1 = T("dt1", j).float()
        ref, s0, s1, sc_ = bn_back(da, T("t1", j).float(), 2 * j, f"{pre}.bn1.weight")
        check_bf16(f"dt1[{j}]", dt1[:, :H], ref, stats, sc_)
        check_rel(f"dbeta1[{j}]", gd[f"{pre}.bn1.bias"], s0)
        check_rel(f"dgamma1[{j}]", gd[f"{pre}.bn1.weight"], s1)
        check_rel(f"dW1[{j}]", gd[f"{pre}.layer1.weight"], dt1[:, :H].double().T @ hs[j][:, :H].double())
        assert gd[f"{pre}.layer1.bias"].abs().max() == 0
        W1 = pad(Wb(f"{pre}.layer1.weight"), Hp, Hp)
        Gj = dt1 @ W1 + du
        Gs = (dt1.abs() @ W1.abs() + du.abs())[:, :H]
        if j > 0:
            check_bf16(f"du[{j - 1}]", T("du", j - 1).float()[:, :H],
                       (Gj * (hs[j] > 0).float())[:, :H], stats, Gs)
        else:
            G = T("G").float()
            check_bf16("G", G[:, :H], Gj[:, :H], stats, Gs)
    check_rel("db0", gd["initial_deep_layer.bias"], G[:, :H].double().sum(0))
    check_rel("dW0", gd["initial_deep_layer.weight"], G[:, :H].double().T @ x0.double())
    Dq = (Dp + 31) // 32 * 32
    dx0 = T("dx0", cols=Dq, dtype=f32)[:, :D]
    check_rel("dx0", dx0, G[:, :H].double() @ W0.double())
    # cross backward (fp64 from the fp32 gathered rows).  The weight gradients'
    # x_0 part is summed over the STORED x0 (bf16 here, like dW0's): x_l enters
    # them as x_l + a_l (x0 - x0f), a_l = prod_{j<l} (1 + s_j)
    dxs = x0.double() - x0f.double()
    a_l = [torch.ones(B, dtype=torch.float64, device=dev)]
    for l in range(Lc):
        a_l.append(a_l[-1] * (1.0 + ss[l]))
    dx = dz.double()[:, None] * wf[H:].double()
    check_rel("dW_f[H:]", gd["final_linear.weight"][0, H:],
              (x + a_l[Lc][:, None] * dxs).T @ dz.double())
    check_rel("db_f", gd["final_linear.bias"], dz.double().sum().reshape(1))
    for l in reversed(range(cfg["params"]["n_cross_layers"])):
        xl, sl = xs[l], ss[l]
        wl = sd0[f"cross_network.{l}.w.weight"][0].double()
        check_rel(f"cross_b[{l}]", gd[f"cross_network.{l}.b"], dx.sum(0))
        gx = (dx * xl).sum(1)
        check_rel(f"cross_w[{l}]", gd[f"cross_network.{l}.w.weight"][0],
                  (gx[:, None] * (xl + a_l[l][:, None] * dxs)).sum(0))
        dx = dx * (1.0 + sl)[:, None] + gx[:, None] * wl[None, :]
    # dx0_cross = sum_k xcoef[b][k] V_k, V = (w_0 .. w_{L-1}, w_f[H:])
    xco = T("xcoef", cols=Lc + 1, dtype=f32).double()
    Vs = [sd0[f"cross_network.{m}.w.weight"][0].double() for m in range(Lc)] + [wf[H:].double()]
    check_rel("dx0_cross", sum(xco[:, k:k + 1] * Vs[k][None] for k in range(Lc + 1)), dx)
    dxe = dx0.double() + dx
    off = 0
    tabs = [("user_embedding.weight", u), ("item_embedding.weight", i)]
    tabs += [(f"cat_embeddings.{k}.weight", c[:, k]) for k in range(K)]
    for name, idx in tabs:
        w = sd0[name].shape[1]
        ref = torch.zeros(sd0[name].shape, dtype=torch.float64, device=dev)
        ref.index_add_(0, idx, dxe[:, off:off + w])
        off += w
        check_rel(name, gd[name], ref)
    print("\n  stage, fraction of elements off by a bf16 rounding flip, max |diff|")
    for name, fr, mx in stats:
        print(f"    {name:10s} {fr:.2e} {mx:.2e}")
