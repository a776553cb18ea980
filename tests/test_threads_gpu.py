"""Re-entrancy of the eval / serving path ("Threading: eval
forward must be re-entrant"): the reference's /recommendations handler is a
sync ``def`` (main.py:306-307), which Starlette runs in its threadpool, so
several requests score the one loaded model at once (main.py:319-322).

Eight host threads score different batches on ONE bf16 model and ONE
RankingPipeline at the same time -- half of them on their own HIP streams,
so kernels of different requests really run concurrently -- and every
result must equal the serial result of the same call bit for bit (the eval
kernels are deterministic: fixed-order sums, no atomics).  Covers the
library's one-time kernel-attribute setup (set_max_dyn_lds, per device under
a lock), the per-call eval workspace, the id-check ring (IndexErrorWatch
slots under a lock) and the per-thread gather_cross error flag.
"""
import threading

import numpy as np
import pytest
import torch

from helpers import our_model

pytestmark = pytest.mark.gpu

CFG = dict(n_users=5000, n_items=3000, cat_dims={"a": 30, "b": 250, "c": 1000}, n_num=4,
           params=dict(emb_dim=16, hidden_dim=128, n_cross_layers=2, n_res_blocks=2,
                       dropout=0.0))
THREADS = 8
REPEAT = 4


def _requests(dev, n_items, item_cat, item_num):
    rng = np.random.default_rng(21)
    reqs = []
    for t in range(THREADS):
        n = 700 + 131 * t
        u = torch.from_numpy(rng.integers(0, CFG["n_users"], n)).to(dev)
        i = torch.from_numpy(rng.integers(0, n_items, n)).to(dev)
        c = torch.from_numpy(np.stack([rng.integers(0, k, n) for k in CFG["cat_dims"].values()],
                                      1)).to(dev)
        x = torch.from_numpy(rng.random((n, CFG["n_num"]), dtype=np.float32)).to(dev)
        pos = rng.choice(n_items, 5 + t, replace=False)
        reqs.append(dict(batch=(u, i, c, x), user=int(rng.integers(0, CFG["n_users"])), pos=pos,
                         lam=(1.0, 0.7, 0.4, 0.0)[t % 4]))
    return reqs


def _run(model, pipe, r):
    with torch.no_grad():
        z = model(*r["batch"])
        cross = model.gather_cross(*r["batch"])
    rows, logits = pipe.recommend(r["user"], r["pos"], lambda_param=r["lam"], top_k=20)
    return z.cpu(), cross.cpu(), rows.cpu(), logits.cpu()


def test_threaded_scoring_equals_serial(dev):
    import dcnr
    model = our_model(CFG, precision="bf16", seed=7).to(dev).eval()
    n_items = CFG["n_items"]
    rng = np.random.default_rng(3)
    item_cat = np.stack([rng.integers(0, k, n_items) for k in CFG["cat_dims"].values()], 1)
    item_num = rng.random((n_items, CFG["n_num"]), dtype=np.float32)
    pipe = dcnr.serving.RankingPipeline(model, item_cat, item_num)
    reqs = _requests(dev, n_items, item_cat, item_num)
    serial = [_run(model, pipe, r) for r in reqs]
    torch.cuda.synchronize()
    model.check_index_errors()

    results = [[None] * REPEAT for _ in range(THREADS)]
    errors = []
    start = threading.Barrier(THREADS)

    def worker(t):
        try:
            own = torch.cuda.Stream(dev) if t % 2 else None
            start.wait()
            for k in range(REPEAT):
                if own is not None:
                    with torch.cuda.stream(own):
                        out = _run(model, pipe, reqs[t])
                else:
                    out = _run(model, pipe, reqs[t])
                results[t][k] = out
        except BaseException as e:   # noqa: BLE001 -- reported by the main thread
            errors.append((t, e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=300)
    assert not any(th.is_alive() for th in ths), "a scoring thread hung"
    assert not errors, errors
    torch.cuda.synchronize()
    model.check_index_errors()
    for t in range(THREADS):
        for k in range(REPEAT):
            for name, a, b in zip(("logits", "cross", "rows", "rank_logits"), results[t][k],
                                  serial[t]):
                assert torch.equal(a, b), (t, k, name)
