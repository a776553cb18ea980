"""Lab: where do the row-map and dense-gradient trainers' moments differ?
(test_row_map_gpu.py::test_fused_trainer_row_map_bit_identical, fp32)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..",
                                "hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd"))
import dcnr  # noqa: E402


def our_model(cfg, precision):
    torch.manual_seed(1234)
    return dcnr.DCN_RecSys(cfg["n_users"], cfg["n_items"], cfg["cat_dims"], cfg["n_num"],
                           dict(cfg["params"]), precision=precision)


def batch(cfg, B, g, dev):
    nu, ni = cfg["n_users"], cfg["n_items"]
    u = torch.randint(0, nu, (B,), generator=g, device=dev)
    i = torch.randint(0, ni, (B,), generator=g, device=dev)
    cd = list(cfg["cat_dims"].values())
    c = torch.stack([torch.randint(0, k, (B,), generator=g, device=dev) for k in cd], 1)
    n = torch.rand((B, cfg["n_num"]), generator=g, device=dev)
    y = (torch.rand(B, generator=g, device=dev) < 0.5).float()
    return u, i, c, n, y


def _segs(t):
    model = t.model
    d = model._dims
    rows = [d['n_users'], d['n_items']] + list(d['cat_dims'])
    offs = model.flat_offsets
    params = model.param_tensors()
    out, pos = [], 0
    for k, r in enumerate(rows):
        if offs[k] > pos:
            out.append((pos, offs[k] - pos, None, 1))
        w = params[k].shape[1]
        out.append((offs[k], r * w, "map", w))
        pos = offs[k] + r * w
    return out


def run(precision, rep):
    dev = torch.device("cuda:0")
    cfg = dict(n_users=20000, n_items=3000, cat_dims={"a": 1000, "b": 37, "c": 250}, n_num=5,
               params=dict(emb_dim=32, hidden_dim=128, n_cross_layers=3, n_res_blocks=2,
                           dropout=0.6))
    m1 = our_model(cfg, precision=precision).to(dev)
    m2 = copy.deepcopy(m1)
    t1 = dcnr.FusedTrainer(m1, lr=1e-3, weight_decay=1e-4)
    t2 = dcnr.FusedTrainer(m2, lr=1e-3, weight_decay=1e-4, dense_table_grads=True)
    g = torch.Generator(device=dev).manual_seed(11)
    bad = []
    for s in range(3):
        b = batch(cfg, 3000, g, dev)
        torch.cuda.manual_seed(100 + s)
        t1.step(*b)
        torch.cuda.manual_seed(100 + s)
        t2.step(*b)
        torch.cuda.synchronize()
        for name, a, c in (("p", t1.flat, t2.flat), ("m", t1.m, t2.m), ("v", t1.v, t2.v),
                           ("g", t1.gflat, t2.gflat)):
            if name == "g":
                continue
            ne = (a != c).nonzero().flatten()
            if ne.numel() and name == "v":
                j = int(ne[0])
                segs = [(lo, c_, mp, w) for lo, c_, mp, w in _segs(t1)]
                print("  step", s, "idx", j, "g1", t1.gflat[j].item(), "g2", t2.gflat[j].item(),
                      "m", t1.m[j].item(), t2.m[j].item(), "p", t1.flat[j].item(),
                      "seg", [sg for sg in segs if sg[0] <= j < sg[0] + sg[1]],
                      "widths", [tuple(x.shape) for x in m1.param_tensors()[:5]], flush=True)
            if ne.numel():
                bad.append((s, name, ne.numel(), ne[:6].tolist(), a[ne[:3]].tolist(), c[ne[:3]].tolist()))
    offs = m1.flat_offsets
    print(f"{precision} rep {rep}: offsets {list(offs)[:6]} E {t1.E} N {t1.flat.numel()}",
          "OK" if not bad else bad, flush=True)
    return not bad


ok = True
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    ok &= run("fp32", rep)
    ok &= run("bf16", rep)
print("ALL OK" if ok else "MISMATCH", os.environ.get("DCNR_LIB", "default lib"))
