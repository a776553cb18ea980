"""GPU parity of the HIP DCN-R path (libdcnr via dcnr.DCN_RecSys) against the
reference's golden fixtures (tests/golden, made by running the reference) and
the fp64 CPU oracle.

Tolerances (measured on the reference itself):
  logits fp32 : |dz| <= 1e-4 * max(|ref|, 1) element-wise vs fp64
  grads fp32  : ||dg|| / ||g64|| <= 5e-3 per tensor (atol 1e-7 for the
                pre-BN Linear biases whose true gradient is ~0)
  gathers     : bit-exact (checked through eval logits of an identity-like model)
  bf16 mode   : logits norm-rel <= 1e-2 vs fp32 oracle
"""
import copy

import numpy as np
import pytest
import torch

import dcnr_oracle as orc
import golden_common as gc
from conftest import golden
from helpers import (assert_grads_close, check_checksums, grad_rel, logits_err, np_state,
                     our_model, spec_of, to_dev)

pytestmark = pytest.mark.gpu


def run_train(model, dev, u, i, c, n, y):
    import dcnr
    model.train()
    model.zero_grad(set_to_none=True)
    z = model(*to_dev(dev, u, i, c, n))
    loss = dcnr.BCEWithLogitsLoss()(z, to_dev(dev, y)[0])
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().double().numpy() for k, p in model.named_parameters()}
    return z.detach().cpu().double().numpy(), float(loss), grads


def test_f1_cfg1_eval_logits(dev):
    fx = golden("f1_cfg1_eval.npz")
    m = our_model(gc.CFG1)
    check_checksums(m, fx)
    m = m.to(dev).eval()
    with torch.no_grad():
        z = m(*to_dev(dev, fx["user"], fx["item"], fx["cat"], fx["num"])).cpu().numpy()
    assert z.shape == (200,)
    assert logits_err(z, fx["logits64"]) <= 1e-4
    assert logits_err(z, fx["logits"]) <= 1e-4


def test_f2_cfg1_train_step(dev):
    fx = golden("f2_cfg1_train.npz")
    m = our_model(gc.CFG1)
    check_checksums(m, fx)
    m = m.to(dev)
    z, loss, grads = run_train(m, dev, fx["user"], fx["item"], fx["cat"], fx["num"], fx["y"])
    assert logits_err(z, fx["logits64"]) <= 1e-4
    assert abs(loss - float(fx["loss64"])) <= 1e-5 * max(1.0, abs(float(fx["loss64"])))
    names = list(fx["names"])
    ref = {}
    for k in names:
        if "embedding" in k:
            full = np.zeros_like(grads[k])
            full[fx["grow:" + k]] = fx["gval:" + k]
            ref[k] = full
        else:
            ref[k] = fx["g:" + k].astype(np.float64)
    assert_grads_close(grads, ref, rtol=5e-3, atol=1e-7)
    # rows never touched have exactly zero gradient (dense embedding grad)
    for k in names:
        if "embedding" in k:
            untouched = np.setdiff1d(np.arange(grads[k].shape[0]), fx["grow:" + k])
            assert np.all(grads[k][untouched] == 0.0), k
    # BN running statistics after one train forward
    sd = {k: v.detach().cpu().double().numpy() for k, v in m.state_dict().items()}
    for k in fx.files:
        if k.startswith("bn:"):
            np.testing.assert_allclose(sd[k[3:]], fx[k], rtol=2e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("opt", ["adamw", "adam"])
def test_f2_cfg1_optimizer_step(dev, opt):
    import dcnr
    fx = golden("f2_cfg1_train.npz")
    m = our_model(gc.CFG1).to(dev)
    run_train(m, dev, fx["user"], fx["item"], fx["cat"], fx["num"], fx["y"])
    # use the reference's own (fp32) gradients so the check isolates the optimizer
    names = list(fx["names"])
    for k, p in m.named_parameters():
        if "embedding" in k:
            g = torch.zeros_like(p)
            g[torch.from_numpy(fx["grow:" + k]).to(dev)] = torch.from_numpy(fx["gval:" + k]).to(dev)
        else:
            g = torch.from_numpy(fx["g:" + k]).to(dev)
        p.grad = g.contiguous()
    cls = dcnr.AdamW if opt == "adamw" else dcnr.Adam
    o = cls(m.parameters(), lr=1e-3, weight_decay=1e-4)
    o.step()
    torch.cuda.synchronize()
    after = {k: p.detach().cpu().double().numpy() for k, p in m.named_parameters()}
    tid, fidx, val = fx[f"{opt}_tid"], fx[f"{opt}_fidx"], fx[f"{opt}_val"]
    got = np.array([after[names[t]].reshape(-1)[f] for t, f in zip(tid, fidx)])
    np.testing.assert_allclose(got, val, rtol=1e-5, atol=2e-7)
    sums = np.array([after[k].sum() for k in names])
    np.testing.assert_allclose(sums, fx[f"{opt}_sum"], rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("opt", ["adamw", "adam"])
def test_adam_kernel_matches_torch_optim_on_device(dev, opt):
    """dcnr_adam_step follows torch.optim.AdamW / Adam's foreach form (the
    one torch runs on a GPU, train.py:201-204) operation by operation: v*b2
    rounded before the addcmul, the addcdiv as (alpha*m)/denom.
    Not bit for bit: the C ABI carries the betas as fp32, so 1 - b1 and
    1 - b2 are fp32 differences of fp32 betas (1 - 0.999f = 9.9998713e-4),
    where torch rounds its double 1 - 0.999 to fp32 (1.0e-3): about 1 % of
    the parameters differ by an ulp or two after five steps.  Five steps on
    1M random parameters (odd length: the element path for the tail)."""
    import dcnr
    g0 = torch.Generator(device=dev).manual_seed(5)
    n = 1_000_003
    p1 = torch.randn(n, device=dev, generator=g0)
    p2 = torch.nn.Parameter(p1.clone())
    p1 = torch.nn.Parameter(p1)
    cls = dcnr.AdamW if opt == "adamw" else dcnr.Adam
    tcls = torch.optim.AdamW if opt == "adamw" else torch.optim.Adam
    o1 = cls([p1], lr=1e-3, weight_decay=1e-2)
    o2 = tcls([p2], lr=1e-3, weight_decay=1e-2, foreach=True)
    for _ in range(5):
        g = torch.randn(n, device=dev, generator=g0)
        g[::7] = 0.0
        p1.grad, p2.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    torch.cuda.synchronize()
    a, b = p1.detach(), p2.detach()
    same = (a == b).float().mean().item()
    d = (a - b).abs()
    # ~2 ulp of b, or 1e-4 of one update (lr = 1e-3) for parameters near 0
    worst = (d / (b.abs() * 2.4e-7 + 1e-7)).max().item()
    print(f"bit-equal {same:.4f}, max |diff| {d.max().item():.3e}, worst / (2 ulp + 1e-7) {worst:.3f}")
    assert same >= 0.97 and worst <= 1.0, (same, worst)


@pytest.mark.parametrize("fname,cfg", [("f3_cfg3r_train.npz", gc.CFG3R),
                                       ("f3b_odd_train.npz", gc.CFG_ODD)])
def test_f3_train_golden(dev, fname, cfg):
    fx = golden(fname)
    m = our_model(cfg)
    check_checksums(m, fx)
    m = m.to(dev)
    z, loss, grads = run_train(m, dev, fx["user"], fx["item"], fx["cat"], fx["num"], fx["y"])
    assert logits_err(z, fx["logits64"]) <= 1e-4
    assert abs(loss - float(fx["loss64"])) <= 1e-5
    names = list(fx["names"])
    gn = np.array([np.linalg.norm(grads[k]) for k in names])
    ref = fx["gnorm64"]
    big = ref > 1e-6
    np.testing.assert_allclose(gn[big], ref[big], rtol=5e-3)
    assert np.all(gn[~big] < 1e-5)
    got = np.array([grads[names[t]].reshape(-1)[f] for t, f in zip(fx["s_tid"], fx["s_fidx"])])
    scale = np.array([ref[t] for t in fx["s_tid"]])
    # per-sample error relative to its tensor's norm (norm-rel criterion, sampled)
    err = np.abs(got - fx["s_val64"])
    ok = (err <= 5e-3 * scale) | (err <= 1e-7)
    assert ok.all(), (err[~ok], scale[~ok])
    sd = {k: v.detach().cpu().double().numpy() for k, v in m.state_dict().items()}
    for k in fx.files:
        if k.startswith("bn:"):
            np.testing.assert_allclose(sd[k[3:]], fx[k], rtol=2e-5, atol=1e-6, err_msg=k)


RANDOM_CFGS = [
    dict(n_users=500, n_items=300, cat_dims={"a": 5, "b": 200, "c": 1000}, n_num=2,
         params=dict(emb_dim=16, hidden_dim=160, n_cross_layers=1, n_res_blocks=1, dropout=0.0)),
    dict(n_users=64, n_items=64, cat_dims={}, n_num=0,
         params=dict(emb_dim=32, hidden_dim=32, n_cross_layers=6, n_res_blocks=4, dropout=0.0)),
    dict(n_users=1000, n_items=50, cat_dims={"x": 2}, n_num=11,
         params=dict(emb_dim=48, hidden_dim=256, n_cross_layers=0, n_res_blocks=2, dropout=0.0)),
    dict(n_users=2000, n_items=700, cat_dims={f"c{k}": 30 + 17 * k for k in range(6)}, n_num=5,
         params=dict(emb_dim=64, hidden_dim=512, n_cross_layers=3, n_res_blocks=3, dropout=0.0)),
]


def relu_margin(cache):
    """Smallest |pre-ReLU| value: below ~1e-5 an fp32 ReLU mask may flip vs
    fp64 (a legitimate rounding difference, the reference fp32 has it too)."""
    vals = [np.abs(a).min() for a in cache.u + cache.r1]
    return float(min(vals)) if vals else 1.0


@pytest.mark.parametrize("ci", range(len(RANDOM_CFGS)))
@pytest.mark.parametrize("B", [2, 37, 300])
def test_random_configs_vs_oracle(dev, ci, B):
    cfg = RANDOM_CFGS[ci]
    spec = spec_of(cfg)
    for attempt in range(8):  # pick inputs with no element within 1e-5 of a ReLU kink
        m = our_model(cfg, seed=100 + ci).to(dev)
        sd = np_state(m)
        u, i, c, n, y = gc.make_inputs(cfg, B, 1000 + B + 7919 * attempt)
        zr, cache = orc.forward(sd, spec, u, i, c, n, train=True)
        if relu_margin(cache) > 1e-5:
            break
    z, loss, grads = run_train(m, dev, u, i, c, n, y)
    lr, dz = orc.bce_with_logits(zr, y)
    gr = orc.backward(sd, spec, cache, dz, u, i, c)
    # B=2: x_hat = +-d/sqrt(d^2+eps) per column is ill-conditioned in fp32
    assert logits_err(z, zr) <= (1e-4 if B > 2 else 1e-2)
    assert abs(loss - lr) <= 1e-5 * max(1.0, abs(lr)) * (1 if B > 2 else 100)
    if B > 2:
        # at B=2 every BN's input-gradient is identically 0 (x_hat = +-1), so
        # upstream grads are pure rounding noise: only forward is compared
        names = [k for k in gr if not (".layer" in k and k.endswith(".bias"))]
        assert_grads_close(grads, gr, rtol=5e-3, atol=1e-6, names=names)
        # pre-BN Linear biases: true gradient ~0 -> absolute check
        for k in gr:
            if ".layer" in k and k.endswith(".bias"):
                assert np.abs(grads[k] - gr[k]).max() < 1e-5 * max(1.0, np.abs(gr[k.replace(
                    "bias", "weight")]).max()), k
    # eval with the updated running stats
    m.eval()
    with torch.no_grad():
        ze = m(*to_dev(dev, u, i, c, n)).reshape(-1).cpu().numpy()
    zer, _ = orc.forward(sd, spec, u, i, c, n, train=False)
    assert logits_err(ze, zer) <= 1e-4


def test_bf16_mode_close(dev):
    fx = golden("f3_cfg3r_train.npz")
    m = our_model(gc.CFG3R, precision="bf16").to(dev)
    z, loss, grads = run_train(m, dev, fx["user"], fx["item"], fx["cat"], fx["num"], fx["y"])
    ref = fx["logits64"]
    assert np.linalg.norm(z - ref) / np.linalg.norm(ref) <= 1e-2
    assert abs(loss - float(fx["loss64"])) <= 1e-2
    names = list(fx["names"])
    gn = np.array([np.linalg.norm(grads[k]) for k in names])
    big = fx["gnorm64"] > 1e-3
    np.testing.assert_allclose(gn[big], fx["gnorm64"][big], rtol=5e-2)


def test_bf16_eval_fused_close(dev):
    """bf16 eval forward: BatchNorm (running stats) + ReLU (+ residual) run in
    the streaming GEMM epilogue (NT_EPI_BN_RELU / NT_EPI_BN_RESID_RELU);
    checked against the fp64 oracle after a train step moved the running
    stats off their init values."""
    fx = golden("f3_cfg3r_train.npz")
    m = our_model(gc.CFG3R, precision="bf16").to(dev)
    run_train(m, dev, fx["user"], fx["item"], fx["cat"], fx["num"], fx["y"])
    m.eval()
    with torch.no_grad():
        ze = m(*to_dev(dev, fx["user"], fx["item"], fx["cat"], fx["num"])).reshape(-1).cpu().numpy()
    zr, _ = orc.forward(np_state(m), spec_of(gc.CFG3R), fx["user"], fx["item"], fx["cat"], fx["num"],
                        train=False)
    assert np.linalg.norm(ze - zr) / np.linalg.norm(zr) <= 1e-2


def test_batch_one_semantics(dev):
    cfg = gc.CFG_ODD
    m = our_model(cfg).to(dev)
    u, i, c, n, y = gc.make_inputs(cfg, 1, 5)
    m.eval()
    with torch.no_grad():
        z = m(*to_dev(dev, u, i, c, n))
    assert z.dim() == 0
    zr, _ = orc.forward(np_state(m), spec_of(cfg), u, i, c, n, train=False)
    assert logits_err([float(z)], zr) <= 1e-4
    m.train()
    with pytest.raises(ValueError):
        m(*to_dev(dev, u, i, c, n))


def test_eval_rows_independent_full_size_bf16(dev):
    """Full cfg3 model (1M x 32 user table, 100k items, 12 x 1000, D=456, H=512)
    at B=131072 in eval mode: rows are independent, so a sample of rows is
    checked against the fp64 oracle run on those rows only."""
    import dcnr
    cfg = dict(n_users=1_000_000, n_items=100_000, cat_dims={f"c{k}": 1000 for k in range(12)},
               n_num=8, params=dict(emb_dim=32, hidden_dim=512, n_cross_layers=3, n_res_blocks=4,
                                    dropout=0.6))
    for prec, tol in (("fp32", 1e-4), ("bf16", 3e-2)):
        torch.manual_seed(7)
        m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                            dict(cfg["params"]), precision=prec)
        gc.perturb_state(m, 8)
        m = m.to(dev).eval()
        B = 131072
        u, i, c, n, _ = gc.make_inputs(cfg, B, 9)
        with torch.no_grad():
            z = m(*to_dev(dev, u, i, c, n)).cpu().numpy()
        rows = np.random.default_rng(0).choice(B, 64, replace=False)
        sd = np_state(m)
        zr, _ = orc.forward(sd, spec_of(cfg), u[rows], i[rows], c[rows], n[rows], train=False)
        if prec == "fp32":
            assert logits_err(z[rows], zr) <= tol
        else:
            assert np.linalg.norm(z[rows] - zr) / np.linalg.norm(zr) <= tol
        del m
        torch.cuda.empty_cache()


def test_index_out_of_range_raises(dev):
    import dcnr
    cfg = gc.CFG_ODD
    torch.manual_seed(0)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), check_indices=True).to(dev).eval()
    u, i, c, n, _ = gc.make_inputs(cfg, 8, 3)
    u = u.copy()
    u[3] = cfg["n_users"]  # one past the end
    # default: asynchronous, as the reference on cuda (a later call / check raises)
    with torch.no_grad(), pytest.raises(IndexError):
        m(*to_dev(dev, u, i, c, n))
        m.check_index_errors()
    # "sync": the call itself raises
    m.check_indices = "sync"
    with torch.no_grad(), pytest.raises(IndexError):
        m(*to_dev(dev, u, i, c, n))
    u[3] = 0
    with torch.no_grad():
        m(*to_dev(dev, u, i, c, n))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_index_out_of_range_raises_train(dev, precision):
    """Train mode: FusedTrainer's step with an out-of-range id raises
    IndexError through the deferred check (the forward's error word stored
    into the pinned ring slot by the one-wave mirror kernel after its last
    launch); steps with valid ids afterwards (past the ring's in-flight
    depth, so slots recycle) raise nothing."""
    import dcnr
    cfg = gc.CFG3R
    m = our_model(cfg, precision).to(dev)
    t = dcnr.FusedTrainer(m, lr=1e-3, weight_decay=1e-4, optimizer_name="AdamW")
    u, i, c, n, y = gc.make_inputs(cfg, 512, 77)
    c = c.copy()
    c[5, 3] = 1000   # one past the end of a 1000-row categorical table
    with pytest.raises(IndexError):
        t.step(*to_dev(dev, u, i, c, n, y))
        t.check_indices()
    c[5, 3] = 0
    for _ in range(12):
        t.step(*to_dev(dev, u, i, c, n, y))
    t.check_indices()


def test_backward_deterministic(dev):
    """Two backward passes on the same state and batch are bit-identical for
    EVERY gradient, the embedding tables included (csrc/embed_bwd.hip)."""
    cfg = gc.CFG3R
    m = our_model(cfg).to(dev)
    u, i, c, n, y = gc.make_inputs(cfg, 512, 77)
    m2 = copy.deepcopy(m)
    _, _, g1 = run_train(m, dev, u, i, c, n, y)
    _, _, g2 = run_train(m2, dev, u, i, c, n, y)
    for k in g1:   # embedding grads included (sorted, fixed-order sums)
        assert np.array_equal(g1[k], g2[k]), k


def test_dropout_train_step_exact_masks(dev):
    """p=0.6 (the reference's chosen dropout, Documentation.md:219): the GPU
    forward and backward use the counter-based mask of (seed, block, row, col);
    the oracle is fed the same masks (host replica of the hash), so logits,
    loss and every gradient must match the fp64 oracle."""
    import dcnr
    from helpers import dropout_mask_np
    cfg = dict(gc.CFG_ODD, params=dict(gc.CFG_ODD["params"], dropout=0.6))
    spec = spec_of(cfg)
    m = our_model(cfg).to(dev)
    sd = np_state(m)
    B = 256
    u, i, c, n, y = gc.make_inputs(cfg, B, 21)
    from dcnr.model import dropout_seed
    torch.manual_seed(1234)
    seed = dropout_seed(dev, advance=False)   # what forward will draw
    z, loss, grads = run_train(m, dev, u, i, c, n, y)
    masks = [dropout_mask_np(seed, j, B, spec.hidden, 0.6) for j in range(spec.n_res)]
    assert 0.3 < masks[0].mean() < 0.5
    zr, cache = orc.forward(sd, spec, u, i, c, n, train=True, dropout_masks=masks)
    lr, dz = orc.bce_with_logits(zr, y)
    gr = orc.backward(sd, spec, cache, dz, u, i, c)
    assert logits_err(z, zr) <= 1e-4
    assert abs(loss - lr) <= 1e-5
    names = [k for k in gr if not (".layer" in k and k.endswith(".bias"))]
    assert_grads_close(grads, gr, rtol=5e-3, atol=1e-6, names=names)


def test_fused_trainer_matches_autograd_adamw(dev):
    """FusedTrainer (flat buffers, one Adam launch) == autograd + dcnr.AdamW."""
    import dcnr
    cfg = gc.CFG3R
    m1 = our_model(cfg).to(dev)
    m2 = copy.deepcopy(m1)
    t = dcnr.FusedTrainer(m1, lr=1e-3, weight_decay=1e-4, optimizer_name="AdamW")
    o = dcnr.AdamW(m2.parameters(), lr=1e-3, weight_decay=1e-4)
    for s in range(1):
        u, i, c, n, y = to_dev(dev, *gc.make_inputs(cfg, 512, 50 + s))
        l1 = t.step(u, i, c, n, y)
        torch.manual_seed(0)
        m2.train()
        o.zero_grad(set_to_none=True)
        l2 = dcnr.BCEWithLogitsLoss()(m2(u, i, c, n), y)
        l2.backward()
        o.step()
        assert abs(float(l1) - float(l2)) < 1e-5
    torch.cuda.synchronize()
    # Adam turns rounding-level gradient differences on (near-)zero gradients
    # (e.g. embedding rows whose contributions cancel; fp32 atomics order)
    # into lr-sized steps: require 99.99% of elements within 1e-4 relative and
    # every element within 3 steps x lr.
    for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        a = a.cpu().double().numpy()
        b = b.cpu().double().numpy()
        close = np.abs(a - b) <= 1e-6 + 1e-4 * np.abs(b)
        if not (".layer" in k and k.endswith(".bias")):  # pre-BN biases: gradient is noise
            assert close.mean() >= 0.999, (k, close.mean())
        assert np.abs(a - b).max() <= 3 * 1e-3 + 1e-6, k


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_training_reduces_loss(dev, precision):
    """A learnable synthetic target (label = sign of a fixed user/item score):
    50 fused steps must reduce the loss and stay finite (bf16 + dropout 0.6)."""
    import dcnr
    cfg = dict(n_users=5000, n_items=2000, cat_dims={f"c{k}": 100 for k in range(4)}, n_num=4,
               params=dict(emb_dim=32, hidden_dim=256, n_cross_layers=3, n_res_blocks=2,
                           dropout=0.6))
    torch.manual_seed(3)
    m = dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                        dict(cfg["params"]), precision=precision).to(dev)
    tr = dcnr.FusedTrainer(m, lr=3e-3, weight_decay=1e-4)
    g = torch.Generator(device=dev).manual_seed(0)
    losses = []
    for s in range(60):
        B = 4096
        u = torch.randint(0, cfg["n_users"], (B,), device=dev, generator=g)
        i = torch.randint(0, cfg["n_items"], (B,), device=dev, generator=g)
        c = torch.randint(0, 100, (B, 4), device=dev, generator=g)
        n = torch.rand((B, 4), device=dev, generator=g)
        y = ((n[:, 0] + 0.3 * (c[:, 1] < 50).float()) > 0.65).float()   # learnable target
        losses.append(float(tr.step(u, i, c, n, y)))
    assert all(np.isfinite(losses))
    assert np.mean(losses[-5:]) < 0.7 * np.mean(losses[:5]), losses


def test_sync_bn_hook_world1_matches_local_bn(dev):
    """SyncBN path (hook between the BN reductions and their consumers, RCCL
    all-reduce of the fp64 statistics) at world size 1 must reproduce local
    BN: same logits, grads and running stats; 4 hook calls per residual block."""
    import socket
    import torch.distributed as dist
    import dcnr
    from dcnr import parallel
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        cfg = gc.CFG3R
        m1 = our_model(cfg).to(dev)
        m2 = copy.deepcopy(m1)
        hook = parallel.install_sync_bn(m2)
        u, i, c, n, y = gc.make_inputs(cfg, 777, 31)
        z1, l1, g1 = run_train(m1, dev, u, i, c, n, y)
        z2, l2, g2 = run_train(m2, dev, u, i, c, n, y)
        R = cfg["params"]["n_res_blocks"]
        assert hook.calls == 4 * R
        np.testing.assert_allclose(z2, z1, rtol=1e-6, atol=1e-6)
        assert abs(l1 - l2) <= 1e-6
        for k in g1:
            np.testing.assert_allclose(g2[k], g1[k], rtol=1e-4, atol=1e-6, err_msg=k)
        for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
            np.testing.assert_allclose(b.cpu().double().numpy(), a.cpu().double().numpy(),
                                       rtol=1e-6, atol=1e-7, err_msg=k)
    finally:
        dist.destroy_process_group()


def test_cosine_knn_vs_sklearn_golden(dev):
    """dcnr.NearestNeighbors (cosine, brute) vs the reference's sklearn index
    (main.py:268-270, 200, 300) on the planted-ties table of F6."""
    import dcnr
    fx = golden("f6_knn.npz")
    table, q_rows = gc.knn_table()
    nn_ = dcnr.NearestNeighbors(metric="cosine", algorithm="brute").fit(table)
    for k in (11, 51):
        d, i = nn_.kneighbors(table[q_rows], n_neighbors=k)
        np.testing.assert_allclose(d, fx[f"d{k}"], rtol=0, atol=2e-6)
        for r in range(len(q_rows)):
            ref_d, ref_i = fx[f"d{k}"][r], fx[f"i{k}"][r]
            inner = ref_d < ref_d[-1] - 2e-6
            assert set(ref_i[inner]) <= set(i[r].tolist())
            # same position for every neighbour not within fp32 noise of another
            near = np.diff(ref_d) <= 2e-6
            isolated = np.ones(k, bool)
            isolated[1:] &= ~near
            isolated[:-1] &= ~near
            np.testing.assert_array_equal(i[r][isolated], ref_i[isolated])


@pytest.mark.parametrize("Q,d", [(1, 64), (3, 64), (8, 64), (32, 64), (256, 64), (64, 32), (600, 64)])
def test_cosine_knn_full_size(dev, Q, d):
    """configs[4] size: cosine top-11 over 1M x d (the bf16-MFMA coarse scan
    + exact fp32 rescoring of its admitted rows, knn.hip scan v4, for every Q)
    against a brute-force torch fp32 reference on the device (random table:
    no ties)."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(11 + Q + d)
    table = torch.randn(1_000_000, d, device=dev, generator=g)
    q = torch.randn(Q, d, device=dev, generator=g)
    nn_ = dcnr.NearestNeighbors(metric="cosine", algorithm="brute").fit(table)
    d, i = nn_.kneighbors(q, n_neighbors=11)
    d = np.asarray(d.cpu() if torch.is_tensor(d) else d)
    i = np.asarray(i.cpu() if torch.is_tensor(i) else i)
    tn = table / table.norm(dim=1, keepdim=True)
    qn = q / q.norm(dim=1, keepdim=True)
    ref_d, ref_i = torch.topk(1.0 - qn @ tn.T, 11, dim=1, largest=False)
    ref_d, ref_i = ref_d.cpu().numpy(), ref_i.cpu().numpy()
    np.testing.assert_allclose(d, ref_d, rtol=0, atol=2e-6)
    for r in range(Q):
        near = np.diff(ref_d[r]) <= 2e-6
        isolated = np.ones(11, bool)
        isolated[1:] &= ~near
        isolated[:-1] &= ~near
        np.testing.assert_array_equal(i[r][isolated], ref_i[r][isolated])


@pytest.mark.parametrize("d", [32, 64])
def test_cosine_pack_rows_and_packed_scan(dev, d):
    """dcnr_cosine_pack_rows = bf16(x * inv_norm) bit for bit (torch's
    round-to-nearest-even cast of the same fp32 product), and the top-k read
    through the packed copy equals the top-k without it, bit for bit, for
    every query-batch shape scan v4 dispatches (NQB 2 .. 16, a partial tail)."""
    import dcnr
    from dcnr import _lib
    g = torch.Generator(device=dev).manual_seed(40 + d)
    table = torch.randn(300_000, d, device=dev, generator=g)
    table[7] = 0.0   # zero row: inv norm 1 (sklearn's normalize)
    nn_ = dcnr.NearestNeighbors(metric="cosine").fit(table)
    assert nn_._packed is not None
    ref = (table * nn_._inv[:, None]).to(torch.bfloat16).view(torch.int16)
    assert torch.equal(nn_._packed, ref)
    for Q in (16, 50, 128, 256, 300):
        q = torch.randn(Q, d, device=dev, generator=g)
        dp, ip = nn_.kneighbors_device(q, 11)
        packed, nn_._packed = nn_._packed, None
        try:
            du, iu = nn_.kneighbors_device(q, 11)
        finally:
            nn_._packed = packed
        assert torch.equal(ip, iu), Q
        assert torch.equal(dp, du), Q
    lib = _lib.load()
    bad = torch.empty((10, 12), dtype=torch.int16, device=dev)
    assert lib.dcnr_cosine_pack_rows(table.data_ptr(), nn_._inv.data_ptr(), 10, 12, bad.data_ptr(),
                                     _lib.stream_ptr(dev)) != 0   # d % 8 != 0


@pytest.mark.parametrize("d,k", [(64, 32), (32, 11), (64, 1), (64, 64)])
def test_cosine_knn_v4_ties_zero_rows_and_kmax(dev, d, k):
    """Scan v4 edge cases (ties, nulls, maximum k): 40 exact
    copies of row 5 scattered over the table (one distance for all 41, so
    ordered by row index), all-zero rows (sklearn's normalize leaves them
    zero: distance 1 to every query), a zero query (distance 1 to every row:
    the k lowest rows; its list overflows scan v4 and takes the exact path),
    k up to v4's 32 and KMAX = 64 (the exact scan); the rest of every list
    against a torch fp32 brute force."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(77 + d + k)
    N = 120_000
    table = torch.randn(N, d, device=dev, generator=g)
    dup = torch.randperm(N, device=dev, generator=g)[:40]
    dup = dup[dup != 5]
    table[dup] = table[5].clone()
    zero = torch.randperm(N, device=dev, generator=g)[:25]
    zero = zero[(zero != 5) & ~torch.isin(zero, dup)]
    table[zero] = 0.0
    nn_ = dcnr.NearestNeighbors(metric="cosine").fit(table)
    q = torch.cat([table[5:6] * 3.0, torch.randn(6, d, device=dev, generator=g)])
    dist_, idx = nn_.kneighbors_device(q, k)
    dist_, idx = dist_.cpu().numpy(), idx.cpu().numpy()
    # query 0: the 41 rows on its direction first, ascending rows, one distance
    ties = np.sort(np.concatenate([[5], dup.cpu().numpy()]))
    m = min(k, ties.size)
    assert idx[0][:m].tolist() == ties[:m].tolist()
    assert np.all(dist_[0][:m] == dist_[0][0]) and dist_[0][0] <= 2e-6
    # random queries: against torch fp32 (zero rows at distance 1)
    tn = table / table.norm(dim=1, keepdim=True).clamp_min(1e-30)
    qn = q[1:] / q[1:].norm(dim=1, keepdim=True)
    ref_d, ref_i = torch.topk((1.0 - qn @ tn.T).clamp(0, 2), k, dim=1, largest=False)
    ref_d, ref_i = ref_d.cpu().numpy(), ref_i.cpu().numpy()
    np.testing.assert_allclose(dist_[1:], ref_d, rtol=0, atol=2e-6)
    for r in range(ref_d.shape[0]):
        near = np.diff(ref_d[r]) <= 2e-6
        iso = np.ones(k, bool)
        iso[1:] &= ~near
        iso[:-1] &= ~near
        np.testing.assert_array_equal(idx[1 + r][iso], ref_i[r][iso])
    # every list sorted by (distance, row)
    for r in range(idx.shape[0]):
        key = list(zip(dist_[r].tolist(), idx[r].tolist()))
        assert key == sorted(key)
    # the zero query: every distance is 1 -> rows 0 .. k-1
    dz, iz = nn_.kneighbors_device(torch.zeros(1, d, device=dev), k)
    assert iz.cpu().numpy()[0].tolist() == list(range(k))
    assert np.all(dz.cpu().numpy() == 1.0)


@pytest.mark.parametrize("N,d", [(100_000, 64), (50_000, 32)])
def test_cosine_knn_v2_v4_same_answer(dev, N, d):
    """One query alone takes scan v2 on these tables; the same query in a
    batch of 2 / 40 takes scan v4 (coarse bf16 admission + exact rescoring):
    rows and distances bit-identical (v4's exact distances use v2's
    arithmetic), so the scan a shape happens to take never changes an
    answer."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(9 + d)
    table = torch.randn(N, d, device=dev, generator=g)
    q = torch.randn(40, d, device=dev, generator=g)
    nn_ = dcnr.NearestNeighbors(metric="cosine").fit(table)
    for r in range(3):
        d1, i1 = nn_.kneighbors_device(q[r:r + 1], 11)
        d2, i2 = nn_.kneighbors_device(q[r:r + 2], 11)
        d40, i40 = nn_.kneighbors_device(q, 11)
        assert torch.equal(i1[0], i2[0]) and torch.equal(d1[0], d2[0]), r
        assert torch.equal(i1[0], i40[r]) and torch.equal(d1[0], d40[r]), r


@pytest.mark.parametrize("N,Q,d", [(11, 2, 64), (12, 40, 32), (600, 3, 64), (5633, 33, 64),
                                   (65537, 17, 32), (70001, 40, 64), (3001, 5, 36), (65536, 1, 64)])
def test_cosine_knn_small_and_ragged_tables(dev, N, Q, d):
    """Ragged shapes around scan v4's fixed sizes (empty / ragged
    inputs): tables of exactly k rows, fewer than k bound blocks of B5_C rows
    (the admission bound is then +inf and every row is rescored exactly),
    one row past the V4_S bound sample, row counts that are no multiple of any
    block size, query counts that straddle the 16-query MFMA tile and the
    32-query in-scan merge, a d that takes scan v2 (36), and a single query
    (scan v2 below V4_Q1_N rows): every list against a torch fp32 brute force,
    sorted by (distance, row)."""
    import dcnr
    k = 11
    g = torch.Generator(device=dev).manual_seed(N + Q + d)
    table = torch.randn(N, d, device=dev, generator=g)
    q = torch.randn(Q, d, device=dev, generator=g)
    nn_ = dcnr.NearestNeighbors(metric="cosine").fit(table)
    dist_, idx = nn_.kneighbors_device(q, k)
    dist_, idx = dist_.cpu().numpy(), idx.cpu().numpy()
    tn = table / table.norm(dim=1, keepdim=True)
    qn = q / q.norm(dim=1, keepdim=True)
    ref_d, ref_i = torch.topk(1.0 - qn @ tn.T, k, dim=1, largest=False)
    ref_d, ref_i = ref_d.cpu().numpy(), ref_i.cpu().numpy()
    np.testing.assert_allclose(dist_, ref_d, rtol=0, atol=2e-6)
    for r in range(Q):
        near = np.diff(ref_d[r]) <= 2e-6
        iso = np.ones(k, bool)
        iso[1:] &= ~near
        iso[:-1] &= ~near
        np.testing.assert_array_equal(idx[r][iso], ref_i[r][iso])
        key = list(zip(dist_[r].tolist(), idx[r].tolist()))
        assert key == sorted(key)
    if N == k:   # every row, in distance order
        assert all(sorted(row) == list(range(N)) for row in idx.tolist())
    d0, i0 = nn_.kneighbors_device(q[:0], k)   # no queries: empty lists
    assert tuple(d0.shape) == (0, k) and tuple(i0.shape) == (0, k)
    with pytest.raises(ValueError):   # sklearn's check_array on the host API
        nn_.kneighbors(np.zeros((0, d), np.float32), n_neighbors=k)
    if N < 64:   # sklearn's error for n_neighbors > n_samples_fit
        with pytest.raises(ValueError):
            nn_.kneighbors_device(q, N + 1)


@pytest.mark.parametrize("Q,dim", [(32, 64), (256, 64), (40, 32), (2, 64), (16, 32)])
def test_cosine_knn_v4_overflow_falls_back_exact(dev, Q, dim):
    """More than V4_CAP rows inside one query's admission bound (12000 rows
    on the query's own direction, every one at distance 0): scan v4's list
    overflows and that query is answered by the exact per-query scan inside
    its rescore block (knn.hip exact_query_topk): the exact top-k, ties by
    row index (the duplicates' lowest rows); every other query of the batch
    keeps the v4 answer, checked against torch fp32."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(5 + Q + dim)
    table = torch.randn(200_000, dim, device=dev, generator=g)
    q = torch.randn(Q, dim, device=dev, generator=g)
    dup = torch.randperm(200_000, device=dev, generator=g)[:12000]
    table[dup] = q[0] * 2.0
    nn_ = dcnr.NearestNeighbors(metric="cosine", algorithm="brute").fit(table)
    d, i = nn_.kneighbors(q, n_neighbors=11)
    assert np.all(d[0] <= 2e-6)
    assert i[0].tolist() == sorted(dup.cpu().tolist())[:11]
    tn = table / table.norm(dim=1, keepdim=True)
    qn = q / q.norm(dim=1, keepdim=True)
    ref_d, ref_i = torch.topk(1.0 - qn @ tn.T, 11, dim=1, largest=False)
    ref_d, ref_i = ref_d.cpu().numpy(), ref_i.cpu().numpy()
    np.testing.assert_allclose(d[1:], ref_d[1:], rtol=0, atol=2e-6)
    for r in range(1, Q):
        near = np.diff(ref_d[r]) <= 2e-6
        isolated = np.ones(11, bool)
        isolated[1:] &= ~near
        isolated[:-1] &= ~near
        np.testing.assert_array_equal(i[r][isolated], ref_i[r][isolated])


@pytest.mark.parametrize("Q,dim", [(3, 64), (16, 64), (5, 32)])
def test_cosine_knn_v4_all_overflow_split_fallback(dev, Q, dim):
    """Every query overflows (6000 duplicates of each query's direction):
    with few queries (Q <= 16) the exact fallback is split over up to 64
    blocks per query, each scanning a slice of the table, the last one
    merging the k-lists (knn.hip rescore_kernel).  Each query's answer is
    its exact top-k -- the 11 lowest duplicate rows at distance 0 -- and the
    answers equal the unsplit single-block fallback's (the same query
    answered inside a batch of 32, where the fallback is not split)."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(17 + Q + dim)
    n = 120_000 + 6000 * Q
    table = torch.randn(n, dim, device=dev, generator=g)
    q = torch.randn(32, dim, device=dev, generator=g)
    perm = torch.randperm(n, device=dev, generator=g)
    dups = [perm[6000 * j:6000 * (j + 1)] for j in range(Q)]
    for j in range(Q):
        table[dups[j]] = q[j] * (1.0 + j)
    nn_ = dcnr.NearestNeighbors(metric="cosine", algorithm="brute").fit(table)
    d, i = nn_.kneighbors(q[:Q], n_neighbors=11)
    d32, i32 = nn_.kneighbors(q, n_neighbors=11)   # 32 queries: one fallback block per query
    for j in range(Q):
        assert np.all(d[j] <= 2e-6)
        assert i[j].tolist() == sorted(dups[j].cpu().tolist())[:11]
    assert np.array_equal(i, i32[:Q]) and np.array_equal(d, d32[:Q])


@pytest.mark.parametrize("Q,dim,every", [(40, 64, 3), (256, 64, 4), (256, 32, 1), (17, 64, 1)])
def test_cosine_knn_v4_batched_fallback(dev, Q, dim, every):
    """Q > 16 with some (every-th) or all queries overflowing (5000
    duplicates of their direction): the batched exact fallback -- groups of 8
    queries x row chunks, each chunk read once per group, per-group
    last-arriver merge (knn.hip exact_batch_item) -- returns each overflowed
    query's 11 lowest duplicate rows, and the whole answer equals the same
    queries asked 16 at a time (the split fallback and the unchanged
    per-query path), bit for bit."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(31 + Q + dim + every)
    over = list(range(0, Q, every))
    n = 150_000 + 5000 * len(over)
    table = torch.randn(n, dim, device=dev, generator=g)
    q = torch.randn(Q, dim, device=dev, generator=g)
    perm = torch.randperm(n, device=dev, generator=g)
    dups = {j: perm[5000 * t:5000 * (t + 1)] for t, j in enumerate(over)}
    for j, rr in dups.items():
        table[rr] = q[j] * (0.5 + j % 3)
    nn_ = dcnr.NearestNeighbors(metric="cosine", algorithm="brute").fit(table)
    d, i = nn_.kneighbors(q, n_neighbors=11)
    for j, rr in dups.items():
        assert np.all(d[j] <= 2e-6), j
        assert i[j].tolist() == sorted(rr.cpu().tolist())[:11], j
    parts = [nn_.kneighbors(q[a:a + 16], n_neighbors=11) for a in range(0, Q, 16)]
    assert np.array_equal(i, np.concatenate([p[1] for p in parts]))
    assert np.array_equal(d, np.concatenate([p[0] for p in parts]))


@pytest.mark.parametrize("Q,ndup", [(32, 300), (256, 3000), (2, 4000)])
def test_cosine_knn_v4_crowded_bin_sorted(dev, Q, ndup):
    """Hundreds to thousands of rows tied at the k-th distance (duplicates
    of each query's direction, fewer than the list's 4096 slots): the
    rescore block sorts all of them by (distance, row) -- round 5 sent a bin
    of more than 256 rows to the exact whole-table scan -- and returns the
    exact top-k: each query's 11 lowest duplicate rows."""
    import dcnr
    g = torch.Generator(device=dev).manual_seed(23 + Q)
    n = 900_000
    table = torch.randn(n, 64, device=dev, generator=g)
    q = torch.randn(Q, 64, device=dev, generator=g)
    rows = torch.randperm(n, device=dev, generator=g)[:Q * ndup].view(Q, ndup)
    for j in range(Q):
        table[rows[j]] = q[j]
    nn_ = dcnr.NearestNeighbors(metric="cosine", algorithm="brute").fit(table)
    d, i = nn_.kneighbors(q, n_neighbors=11)
    want = torch.sort(rows, dim=1).values[:, :11].cpu().numpy()
    assert np.array_equal(i, want)
    assert np.all(d <= 2e-6)


@pytest.mark.parametrize("M,K,N,out_f32", [(4096, 512, 512, 0), (1000, 456, 512, 1),
                                           (333, 64, 96, 0), (70000, 128, 256, 1)])
def test_linear_bf16_vs_torch(dev, M, K, N, out_f32):
    """dcnr_linear_bf16 (weight-resident streaming MFMA GEMM) vs a torch fp32
    reference of the same bf16 operands; tolerance = bf16 output rounding."""
    import ctypes
    from dcnr import _lib
    g = torch.Generator(device=dev).manual_seed(M + K + N)
    X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g)
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
    lib = _lib.load()
    _lib.check(lib.dcnr_linear_bf16(X.data_ptr(), K, M, K, W.data_ptr(), K, N, b.data_ptr(),
                                    C.data_ptr(), N, out_f32, _lib.stream_ptr(dev)), "linear")
    ref = X.float() @ W.float().T + b
    err = (C.float() - ref).abs().max().item()
    tol = 1e-3 if out_f32 else 1.6e-2 * ref.abs().max().item()
    assert err <= tol, err


@pytest.mark.parametrize("B,N,K,acc", [(131072, 512, 512, 0), (131072, 512, 456, 1),
                                       (37, 96, 64, 0), (5000, 264, 160, 0)])
def test_linear_wgrad_bf16_vs_torch(dev, B, N, K, acc):
    """dcnr_linear_wgrad_bf16 (256x256 LDS-DMA weight-gradient GEMM + split
    reduction) vs a torch fp32 reference of the same bf16 operands."""
    from dcnr import _lib
    g = torch.Generator(device=dev).manual_seed(B + N + K)
    dY = torch.randn(B, N, device=dev, generator=g).to(torch.bfloat16)
    X = torch.randn(B, K, device=dev, generator=g).to(torch.bfloat16)
    dW = torch.randn(N, K, device=dev, generator=g) if acc else torch.empty(N, K, device=dev)
    base = dW.clone()
    lib = _lib.load()
    ws = torch.empty(lib.dcnr_linear_wgrad_workspace_size(N, K, B), dtype=torch.uint8, device=dev)
    _lib.check(lib.dcnr_linear_wgrad_bf16(dY.data_ptr(), N, X.data_ptr(), K, B, N, K, dW.data_ptr(),
                                          acc, ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev)),
               "wgrad")
    ref = dY.float().t() @ X.float() + (base if acc else 0)
    err = ((dW - ref).norm() / ref.norm()).item()
    assert err <= 1e-5, err


def test_reference_artifacts_score_on_gpu(dev):
    """(f)3: the reference's saved artifacts (F9: final_dcn_model.pth +
    item_embeddings.npy, written by train.py:391-394's code) loaded the way
    main.py:256-270 loads them (weights-only), scored on the GPU on F1's
    inputs: F1's logits (the reference's eval forward of that model)."""
    import os
    import dcnr
    d = os.path.join(os.path.dirname(__file__), "golden", "f9_artifacts")
    cfg = gc.CFG1
    model_dims = (cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"])
    m, emb, index = dcnr.artifacts.load_artifacts(d, model_dims, dict(cfg["params"]), device=dev)
    fx = golden("f1_cfg1_eval.npz")
    with torch.no_grad():
        z = m(*to_dev(dev, fx["user"], fx["item"], fx["cat"], fx["num"])).cpu().numpy()
    assert logits_err(z, fx["logits64"]) <= 1e-4
    assert logits_err(z, fx["logits"]) <= 1e-4
    # the index serves /similar_items on the same table (main.py:296-302)
    dist_, idx = index.kneighbors(emb[:3], n_neighbors=5)
    assert np.array_equal(np.asarray(idx)[:, 0], np.arange(3))
