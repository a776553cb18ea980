"""Generate the golden fixtures by running the REFERENCE code in this container.

Run (build container only; /root/reference is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports /root/reference/train.py (optuna is not installed and is only used
inside ``objective``/``__main__``, so a stub module is placed in sys.modules)
and scikit-learn's NearestNeighbors (what main.py:268-270 calls).  Only data
(inputs and reference outputs) is written to tests/golden/*.npz; weights are
regenerated from seeds (golden_common.py) and pinned by checksums.

Fixtures:
  f1_cfg1_eval.npz    cfg1 eval forward, B=200 (fp32 + fp64 logits)
  f2_cfg1_train.npz   cfg1 train mode p=0, B=512: logits, loss, grads,
                      updated BN running stats, one AdamW and one Adam step
  f3_cfg3r_train.npz  reduced cfg3 (D=456, H=512, 4 res, 3 cross), B=1024:
                      logits, loss, per-tensor grad norms, sampled grads
  f3b_odd_train.npz   odd widths (D=70, H=96, 3 res, 4 cross), B=64
  f4_cross_kat.npz    CrossLayer known-answer test, D=7, B=5
  f5_width_rule.npz   n_cat -> int(sqrt(n_cat)) + 1
  f6_knn.npz          cosine kNN vs sklearn brute, 20k x 64, k=11 and k=51
"""
from __future__ import annotations

import copy
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_common as gc  # noqa: E402

REF = "/root/reference"


def load_reference():
    sys.modules.setdefault("optuna", types.ModuleType("optuna"))
    spec = importlib.util.spec_from_file_location("ref_train", os.path.join(REF, "train.py"))
    mod = importlib.util.module_from_spec(spec)
    cwd = os.getcwd()
    os.chdir("/tmp")
    try:
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    return mod


def sampled(grads: dict, names, n, seed):
    """Sample n (tensor-id, flat-index) pairs deterministically."""
    rng = np.random.default_rng(seed)
    sizes = np.array([grads[k].size for k in names])
    tid = rng.choice(len(names), size=n, p=sizes / sizes.sum())
    fidx = np.array([rng.integers(0, sizes[t]) for t in tid], dtype=np.int64)
    vals = np.array([grads[names[t]].reshape(-1)[i] for t, i in zip(tid, fidx)])
    return tid.astype(np.int64), fidx, vals


def run_train(ref, cfg, B, seed_in, dtype=torch.float32):
    m = gc.build(ref.DCN_RecSys, cfg)
    m = m.to(dtype)
    m.train()
    u, i, c, n, y = gc.make_inputs(cfg, B, seed_in)
    T = lambda a: torch.from_numpy(a)
    z = m(T(u), T(i), T(c), T(n).to(dtype))
    loss = torch.nn.BCEWithLogitsLoss()(z, T(y).to(dtype))
    loss.backward()
    grads = {k: p.grad.detach().double().numpy() for k, p in m.named_parameters()}
    return m, (u, i, c, n, y), z.detach().double().numpy(), float(loss), grads


def main():
    ref = load_reference()
    out = {}

    # ---- F1: cfg1 eval forward, B=200 ------------------------------------
    m = gc.build(ref.DCN_RecSys, gc.CFG1).eval()
    u, i, c, n, y = gc.make_inputs(gc.CFG1, 200, 1)
    with torch.no_grad():
        z32 = m(*(torch.from_numpy(a) for a in (u, i, c, n))).numpy()
        m64 = copy.deepcopy(m).double()
        z64 = m64(*(torch.from_numpy(a) for a in (u, i, c)), torch.from_numpy(n).double()).numpy()
    ck = gc.state_checksums(m)
    np.savez_compressed(os.path.join(HERE, "f1_cfg1_eval.npz"), user=u, item=i, cat=c, num=n,
                        logits=z32, logits64=z64,
                        ck_names=np.array(list(ck.keys())), ck=np.stack(list(ck.values())))
    out["f1"] = z32[:4]

    # ---- F2: cfg1 train, p=0, B=512 --------------------------------------
    m, (u, i, c, n, y), z, loss, grads = run_train(ref, gc.CFG1, 512, 2)
    _, _, z64, loss64, grads64 = run_train(ref, gc.CFG1, 512, 2, torch.float64)
    names = [k for k, _ in m.named_parameters()]
    sd = {k: v.detach().double().numpy() for k, v in m.state_dict().items()}
    dense = [k for k in names if "embedding" not in k]
    emb = [k for k in names if "embedding" in k]
    payload = dict(user=u, item=i, cat=c, num=n, y=y, logits=z, logits64=z64,
                   loss=np.float64(loss), loss64=np.float64(loss64),
                   names=np.array(names))
    for k in dense:
        payload["g:" + k] = grads[k].astype(np.float32)
    for k in emb:
        rows = np.nonzero(np.abs(grads64[k]).sum(axis=1) > 0)[0]
        payload["grow:" + k] = rows
        payload["gval:" + k] = grads[k][rows].astype(np.float32)
    for k in sd:
        if "running" in k or "num_batches" in k:
            payload["bn:" + k] = sd[k]
    payload["gnorm64"] = np.array([np.linalg.norm(grads64[k]) for k in names])
    # one optimizer step of each kind on copies (train.py:201-204, 226)
    for opt_name, opt_cls in (("adamw", torch.optim.AdamW), ("adam", torch.optim.Adam)):
        mm = copy.deepcopy(m)
        for (k, p), (_, p0) in zip(mm.named_parameters(), m.named_parameters()):
            p.grad = p0.grad.clone()
        opt = opt_cls(mm.parameters(), lr=1e-3, weight_decay=1e-4)
        opt.step()
        after = {k: p.detach().double().numpy() for k, p in mm.named_parameters()}
        tid, fidx, vals = sampled(after, names, 4096, 11)
        payload[f"{opt_name}_tid"] = tid
        payload[f"{opt_name}_fidx"] = fidx
        payload[f"{opt_name}_val"] = vals
        payload[f"{opt_name}_sum"] = np.array([after[k].sum() for k in names])
    ck = gc.state_checksums(gc.build(ref.DCN_RecSys, gc.CFG1))
    payload["ck_names"] = np.array(list(ck.keys()))
    payload["ck"] = np.stack(list(ck.values()))
    np.savez_compressed(os.path.join(HERE, "f2_cfg1_train.npz"), **payload)
    out["f2"] = loss

    # ---- F3: reduced cfg3, B=1024, and odd shapes ----------------------------
    for fname, cfg, B, seed in (("f3_cfg3r_train.npz", gc.CFG3R, 1024, 3),
                                ("f3b_odd_train.npz", gc.CFG_ODD, 64, 4)):
        m, (u, i, c, n, y), z, loss, grads = run_train(ref, cfg, B, seed)
        _, _, z64, loss64, grads64 = run_train(ref, cfg, B, seed, torch.float64)
        names = [k for k, _ in m.named_parameters()]
        tid, fidx, vals64 = sampled(grads64, names, 4096, 12)
        vals32 = np.array([grads[names[t]].reshape(-1)[f] for t, f in zip(tid, fidx)])
        ck = gc.state_checksums(gc.build(ref.DCN_RecSys, cfg))
        sd = {k: v.detach().double().numpy() for k, v in m.state_dict().items()}
        payload = dict(user=u, item=i, cat=c, num=n, y=y, logits=z, logits64=z64,
                       loss=np.float64(loss), loss64=np.float64(loss64), names=np.array(names),
                       gnorm=np.array([np.linalg.norm(grads[k]) for k in names]),
                       gnorm64=np.array([np.linalg.norm(grads64[k]) for k in names]),
                       s_tid=tid, s_fidx=fidx, s_val64=vals64, s_val32=vals32,
                       ck_names=np.array(list(ck.keys())), ck=np.stack(list(ck.values())))
        for k in sd:
            if "running" in k:
                payload["bn:" + k] = sd[k]
        np.savez_compressed(os.path.join(HERE, fname), **payload)
        out[fname] = loss

    # ---- F4: CrossLayer KAT ------------------------------------------------
    torch.manual_seed(5)
    cl = ref.CrossLayer(7)
    with torch.no_grad():
        cl.b.copy_(torch.arange(7, dtype=torch.float32) * 0.125 - 0.25)
        cl.w.weight.copy_(torch.tensor([[0.5, -0.25, 0.125, 1.0, -1.0, 0.0, 0.75]]))
    x = (torch.arange(35, dtype=torch.float32).reshape(5, 7) - 17) / 8
    y = cl(x).detach().numpy()
    np.savez_compressed(os.path.join(HERE, "f4_cross_kat.npz"), x=x.numpy(),
                        w=cl.w.weight.detach().numpy()[0], b=cl.b.detach().numpy(), y=y)

    # ---- F5: width rule ----------------------------------------------------
    ns = np.array([1, 2, 3, 4, 9, 15, 16, 17, 250, 961, 1000, 1024], dtype=np.int64)
    widths = []
    for nn_ in ns:
        mm = ref.DCN_RecSys(3, 3, {"a": int(nn_)}, 1, dict(emb_dim=4, hidden_dim=8, n_cross_layers=1,
                                                           n_res_blocks=1, dropout=0.0))
        widths.append(mm.cat_embeddings[0].weight.shape[1])
    np.savez_compressed(os.path.join(HERE, "f5_width_rule.npz"), n=ns, width=np.array(widths))

    # ---- F6: cosine kNN vs sklearn (main.py:268-270, 200, 300) -------------
    from sklearn.neighbors import NearestNeighbors
    table, q_rows = gc.knn_table()
    nn_model = NearestNeighbors(n_neighbors=16, metric="cosine", algorithm="brute").fit(table)
    d11, i11 = nn_model.kneighbors(table[q_rows], n_neighbors=11)
    d51, i51 = nn_model.kneighbors(table[q_rows], n_neighbors=51)
    np.savez_compressed(os.path.join(HERE, "f6_knn.npz"), q_rows=q_rows, d11=d11, i11=i11,
                        d51=d51, i51=i51)
    print({k: (np.asarray(v).tolist() if np.ndim(v) else v) for k, v in out.items()})


if __name__ == "__main__":
    main()
