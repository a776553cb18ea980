"""GPU parity of the serving core (dcnr.serving; serving.hip + knn.hip + the
eval forward) against the reference's MMR golden fixture (f8, made by running
main.py:133-169) and the CPU oracle.

Criteria: candidate sets, ranking batches, sort orders and MMR selections are
integer/index results and must be identical; logits follow the fp32 bar of
test_parity_gpu (1e-4 * max(|ref|, 1)).  Inputs are drawn so that no two
scores or similarities that decide an order lie within fp32 rounding.
"""
import numpy as np
import pytest
import torch

import dcnr_oracle as orc
import golden_common as gc
from conftest import golden
from helpers import np_state, our_model, spec_of

pytestmark = pytest.mark.gpu


def test_mmr_vs_reference_golden(dev):
    from dcnr import serving
    fx = golden("f8_mmr.npz")
    ids_all = fx["ids_all"]
    serving.ml_artifacts.clear()
    serving.ml_artifacts['item_embeddings'] = fx["emb"]
    serving.ml_artifacts['artifacts'] = {'item_id_mapping': {int(i): r for r, i in enumerate(ids_all)}}
    serving.ml_artifacts['device'] = dev
    for s, name in enumerate(fx["names"]):
        ranked = list(zip(fx[f"s{s}_scores"].tolist(), fx[f"s{s}_ids"].tolist()))
        got = serving.rerank_with_mmr(ranked, float(fx[f"s{s}_lam"]), int(fx[f"s{s}_topk"]))
        assert got == fx[f"s{s}_out"].tolist(), str(name)
    assert serving.rerank_with_mmr([], 0.5) == []


@pytest.mark.parametrize("n", [1, 7, 300, 4096, 4097, 20000])
def test_rank_by_score_stable(dev, n):
    """n <= SV_MAX: the LDS bitonic kernel; above: the stable device sort."""
    from dcnr.serving import RankingPipeline
    rng = np.random.default_rng(n)
    s = rng.integers(-20, 20, n).astype(np.float32) / 4   # many exact ties
    pipe = RankingPipeline.__new__(RankingPipeline)
    pipe.device = dev
    order = pipe.rank(torch.from_numpy(s).to(dev)).cpu().numpy()
    assert order.tolist() == orc.rank_by_score(s).tolist()


def make_pipeline(dev, n_items=3000, d=16, seed=0):
    import dcnr
    cfg = dict(n_users=400, n_items=n_items, cat_dims={"a": 30, "b": 250, "c": 1000}, n_num=4,
               params=dict(emb_dim=d, hidden_dim=64, n_cross_layers=2, n_res_blocks=2,
                           dropout=0.0))
    m = our_model(cfg, seed=seed).to(dev)
    rng = np.random.default_rng(seed)
    item_cat = np.stack([rng.integers(0, c, n_items) for c in cfg["cat_dims"].values()], 1)
    item_num = rng.random((n_items, 4), dtype=np.float32)
    pipe = dcnr.serving.RankingPipeline(m, item_cat, item_num)
    return cfg, m, pipe, item_cat, item_num


def test_candidate_union_and_batch(dev):
    from dcnr import _lib  # noqa: F401
    cfg, m, pipe, item_cat, item_num = make_pipeline(dev)
    emb = m.item_embedding.weight.detach().cpu().numpy()
    rng = np.random.default_rng(3)
    pos = rng.choice(cfg["n_items"], 40, replace=False)
    cand = pipe.candidates(pos).cpu().numpy()
    _, idx = orc.cosine_kneighbors(emb, emb[pos], 11)
    assert cand.tolist() == orc.candidate_union(pos, idx).tolist()
    u, i, c, x = pipe.ranking_batch(17, torch.from_numpy(cand).to(dev))
    assert (u.cpu().numpy() == 17).all()
    assert np.array_equal(i.cpu().numpy(), cand)
    assert np.array_equal(c.cpu().numpy(), item_cat[cand])
    assert np.array_equal(x.cpu().numpy(), item_num[cand])
    # /similar_items: kneighbors(n+1)[1:]
    sim = pipe.similar_items(int(pos[0]), 10).cpu().numpy()
    assert sim.tolist() == idx[0, 1:].tolist()


def test_candidate_union_above_capacity(dev):
    """Q*k above SV_MAX (a user with 500 positive hotels, k=11): per-chunk
    unions merged give exactly the one-shot union; MMR above SV_MAX raises."""
    from dcnr.serving import SV_MAX, mmr_positions
    cfg, m, pipe, item_cat, item_num = make_pipeline(dev)
    emb = m.item_embedding.weight.detach().cpu().numpy()
    rng = np.random.default_rng(4)
    pos = rng.choice(cfg["n_items"], 500, replace=False)
    assert pos.size * pipe.n_neighbors > SV_MAX
    cand = pipe.candidates(pos).cpu().numpy()
    _, idx = orc.cosine_kneighbors(emb, emb[pos], 11)
    assert cand.tolist() == orc.candidate_union(pos, idx).tolist()
    rows = torch.arange(SV_MAX + 1, device=dev) % cfg["n_items"]
    with pytest.raises(ValueError):
        mmr_positions(pipe.index._table, pipe.index._inv, rows,
                      torch.zeros(SV_MAX + 1, device=dev), 0.5, 5)


@pytest.mark.parametrize("lam", [1.0, 0.7, 0.3])
def test_recommend_matches_oracle(dev, lam):
    cfg, m, pipe, item_cat, item_num = make_pipeline(dev, seed=5)
    sd = np_state(m)
    spec = spec_of(cfg)
    emb = sd['item_embedding.weight'].astype(np.float32)
    rng = np.random.default_rng(11)
    pos = rng.choice(cfg["n_items"], 12, replace=False)
    user = 123
    rows, logits = pipe.recommend(user, pos, lambda_param=lam, top_k=20)
    # oracle composition of main.py:196-203, 215-230, 319-332
    _, idx = orc.cosine_kneighbors(emb, emb[pos], 11)
    cand = orc.candidate_union(pos, idx)
    n = len(cand)
    z, _ = orc.forward(sd, spec, np.full(n, user), cand, item_cat[cand], item_num[cand],
                       train=False)
    order = orc.rank_by_score(z.astype(np.float32))
    ranked, rz = cand[order], z[order]
    zs = np.sort(z)
    assert np.min(np.diff(zs)) > 1e-5, "inputs must not have near-tied scores"
    if lam < 1.0:
        p = orc.mmr_rerank(emb, ranked, rz.astype(np.float32), lam, 20)
        ranked, rz = ranked[p], rz[p]
    assert rows.cpu().numpy().tolist() == ranked.tolist()
    got = logits.cpu().double().numpy()
    assert np.max(np.abs(got - rz) / np.maximum(np.abs(rz), 1.0)) <= 1e-4
    # host filters (city / negative reviews, main.py:210-212)
    allowed = set(cand[::2].tolist())
    excluded = {int(cand[0])}
    rows2, _ = pipe.recommend(user, pos, 1.0, allowed=allowed, excluded=excluded)
    assert set(rows2.cpu().tolist()) == (allowed - excluded)


def test_device_loader_matches_dataloader(dev):
    """Batches of dcnr.DeviceLoader == TensorDataset + DataLoader(shuffle=True)
    batches (train.py:195-196), bit for bit, including the partial last one."""
    from torch.utils.data import DataLoader, TensorDataset
    import dcnr
    rng = np.random.default_rng(0)
    n, K, F = 1003, 5, 3
    collab = torch.from_numpy(rng.integers(0, 1000, (n, 2)))
    cat = torch.from_numpy(rng.integers(0, 50, (n, K)))
    num = torch.from_numpy(rng.random((n, F), dtype=np.float32))
    y = torch.from_numpy((rng.random(n) < 0.5).astype(np.float32))
    for shuffle in (True, False):
        torch.manual_seed(3)
        ref = list(DataLoader(TensorDataset(collab, cat, num, y), batch_size=128, shuffle=shuffle))
        torch.manual_seed(3)
        got = list(dcnr.DeviceLoader(collab, cat, num, y, batch_size=128, shuffle=shuffle))
        assert len(got) == len(ref) == 8
        for g, r in zip(got, ref):
            for a, b in zip(g, r):
                assert torch.equal(a.cpu(), b)


def test_device_loader_epochs_with_dropout_steps(dev):
    """The reference trains on cuda (train.py:32): its dropout draws from the
    device generator, so the CPU generator -- and with it every epoch's
    DataLoader permutation -- is untouched by the training steps.  Two
    DeviceLoader epochs with dropout-0.6 FusedTrainer steps in between must
    give the batches of two DataLoader(shuffle=True) epochs with no steps."""
    from torch.utils.data import DataLoader, TensorDataset
    import dcnr
    rng = np.random.default_rng(1)
    n = 700
    collab = torch.from_numpy(np.stack([rng.integers(0, 300, n), rng.integers(0, 120, n)], 1))
    cat = torch.from_numpy(rng.integers(0, 40, (n, 2)))
    num = torch.from_numpy(rng.random((n, 3), dtype=np.float32))
    y = torch.from_numpy((rng.random(n) < 0.5).astype(np.float32))
    torch.manual_seed(5)
    ref = [list(DataLoader(TensorDataset(collab, cat, num, y), batch_size=100, shuffle=True))
           for _ in range(2)]
    torch.manual_seed(0)
    m = dcnr.DCN_RecSys(300, 120, {"a": 40, "b": 40}, 3,
                        dict(emb_dim=8, hidden_dim=64, n_cross_layers=2, n_res_blocks=2,
                             dropout=0.6)).to(dev)
    tr = dcnr.FusedTrainer(m, lr=1e-3)
    torch.manual_seed(5)
    loader = dcnr.DeviceLoader(collab, cat, num, y, batch_size=100, shuffle=True)
    for ep in range(2):
        got = []
        for b in loader:
            got.append(b)
            cb, ct, nm, yy = b
            tr.step(cb[:, 0], cb[:, 1], ct, nm, yy)
        assert len(got) == len(ref[ep])
        for g, r in zip(got, ref[ep]):
            for a, b in zip(g, r):
                assert torch.equal(a.cpu(), b)
    tr.check_indices()


def test_fused_trainer_reports_bad_ids(dev):
    """An out-of-range id in a FusedTrainer batch surfaces as IndexError (the
    id check is read back asynchronously and reported by a later step or by
    check_indices())."""
    import dcnr
    torch.manual_seed(0)
    m = dcnr.DCN_RecSys(300, 120, {"a": 40}, 3,
                        dict(emb_dim=8, hidden_dim=64, n_cross_layers=1, n_res_blocks=1,
                             dropout=0.0)).to(dev)
    tr = dcnr.FusedTrainer(m, lr=1e-3)
    B = 64
    u = torch.randint(0, 300, (B,), device=dev)
    i = torch.randint(0, 120, (B,), device=dev)
    c = torch.randint(0, 40, (B, 1), device=dev)
    n = torch.rand((B, 3), device=dev)
    y = (torch.rand(B, device=dev) < 0.5).float()
    tr.step(u, i, c, n, y)
    tr.check_indices()
    c[5, 0] = 40
    with pytest.raises(IndexError):
        tr.step(u, i, c, n, y)
        tr.check_indices()


@pytest.mark.parametrize("n,d,top_k", [(400, 64, 20), (700, 64, 12), (1500, 16, 10),
                                       (3000, 16, 6)])
def test_mmr_lds_and_table_paths(dev, n, d, top_k):
    """dcnr_mmr_rerank stages the candidates' rows in LDS when n*(d+1)+n floats
    fit 152 KiB (400 x 64, 1500 x 16) and re-reads the table otherwise
    (700 x 64, 3000 x 16): both against the rerank_with_mmr restatement, with
    rows absent from the mapping (-1) mixed in."""
    from dcnr import serving
    rng = np.random.default_rng(n + d)
    n_items = 5000
    emb = rng.standard_normal((n_items, d)).astype(np.float32)
    rows = rng.choice(n_items, n, replace=False).astype(np.int64)
    rows[rng.choice(np.arange(1, n), n // 50, replace=False)] = -1
    scores = np.sort(rng.random(n).astype(np.float32))[::-1].copy()
    table = torch.from_numpy(emb).to(dev)
    inv = serving.row_inv_norms(table)
    got = serving.mmr_positions(table, inv, torch.from_numpy(rows), torch.from_numpy(scores),
                                0.7, top_k).cpu().tolist()
    assert got == orc.mmr_rerank(emb, rows.tolist(), scores, 0.7, top_k)
