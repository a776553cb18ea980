"""The CPU oracle (oracle/dcnr_oracle.py) pinned against the reference's own
outputs (tests/golden, written by tests/golden/make_golden.py running the
reference train.py / sklearn).  CPU only: this is what makes the oracle a
trustworthy checker for the GPU parity tests."""
import numpy as np
import pytest

import dcnr_oracle as orc
import golden_common as gc
from conftest import golden
from helpers import np_state, our_model, spec_of


def _oracle_train(cfg, fx):
    m = our_model(cfg)                      # same init as the reference (checksums tested)
    sd = np_state(m)
    spec = spec_of(cfg)
    z, cache = orc.forward(sd, spec, fx["user"], fx["item"], fx["cat"], fx["num"], train=True)
    loss, dz = orc.bce_with_logits(z, fx["y"])
    g = orc.backward(sd, spec, cache, dz, fx["user"], fx["item"], fx["cat"])
    return z, loss, g, sd


def test_f1_eval_logits():
    fx = golden("f1_cfg1_eval.npz")
    sd = np_state(our_model(gc.CFG1))
    z, _ = orc.forward(sd, spec_of(gc.CFG1), fx["user"], fx["item"], fx["cat"], fx["num"])
    np.testing.assert_allclose(z, fx["logits64"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(z, fx["logits"], rtol=0, atol=1e-4)   # reference fp32 run


def test_f2_train_logits_loss_grads_bnstats():
    fx = golden("f2_cfg1_train.npz")
    z, loss, g, sd = _oracle_train(gc.CFG1, fx)
    np.testing.assert_allclose(z, fx["logits64"], rtol=1e-12, atol=1e-12)
    assert abs(loss - float(fx["loss64"])) <= 1e-12
    names = list(fx["names"])
    np.testing.assert_allclose([np.linalg.norm(g[k]) for k in names], fx["gnorm64"], rtol=1e-9,
                               atol=1e-15)
    for k in fx.files:
        if k.startswith("g:"):     # the reference fp32 autograd grads
            ref = fx[k].astype(np.float64)
            scale = max(np.linalg.norm(ref), 1e-30)
            assert np.linalg.norm(g[k[2:]] - ref) <= 5e-3 * scale + 1e-7, k
        if k.startswith("grow:"):  # embedding grads: nonzero rows only
            name = k[5:]
            rows = fx[k]
            nz = np.flatnonzero(np.abs(g[name]).sum(1))
            assert set(nz.tolist()) <= set(rows.tolist()), name
            np.testing.assert_allclose(g[name][rows], fx["gval:" + name], rtol=2e-3, atol=1e-7)
        if k.startswith("bn:"):
            np.testing.assert_allclose(np.asarray(sd[k[3:]], np.float64), fx[k], rtol=1e-5,
                                       atol=1e-7, err_msg=k)  # reference ran fp32


@pytest.mark.parametrize("fname,cfg", [("f3_cfg3r_train.npz", gc.CFG3R),
                                       ("f3b_odd_train.npz", gc.CFG_ODD)])
def test_f3_train_sampled_grads(fname, cfg):
    fx = golden(fname)
    z, loss, g, sd = _oracle_train(cfg, fx)
    np.testing.assert_allclose(z, fx["logits64"], rtol=1e-11, atol=1e-11)
    assert abs(loss - float(fx["loss64"])) <= 1e-11
    names = list(fx["names"])
    np.testing.assert_allclose([np.linalg.norm(g[k]) for k in names], fx["gnorm64"], rtol=1e-8,
                               atol=1e-15)
    got = np.array([g[names[t]].reshape(-1)[f] for t, f in zip(fx["s_tid"], fx["s_fidx"])])
    np.testing.assert_allclose(got, fx["s_val64"], rtol=1e-8, atol=1e-14)
    for k in fx.files:
        if k.startswith("bn:"):
            np.testing.assert_allclose(np.asarray(sd[k[3:]], np.float64), fx[k], rtol=1e-5,
                                       atol=1e-7, err_msg=k)  # reference ran fp32


def test_f4_cross_layer_known_answer():
    fx = golden("f4_cross_kat.npz")
    y, _ = orc.cross_layer(fx["x"].astype(np.float64), fx["w"].astype(np.float64),
                           fx["b"].astype(np.float64))
    np.testing.assert_allclose(y, fx["y"], rtol=1e-6, atol=1e-6)


def test_f6_cosine_knn_vs_sklearn():
    fx = golden("f6_knn.npz")
    table, q_rows = gc.knn_table()
    np.testing.assert_array_equal(q_rows, fx["q_rows"])
    for k in (11, 51):
        d, i = orc.cosine_kneighbors(table, table[q_rows], k)
        np.testing.assert_allclose(d, fx[f"d{k}"], rtol=0, atol=2e-6)
        # identical neighbour lists up to the order of exactly tied distances
        for r in range(len(q_rows)):
            ref_i, ref_d = fx[f"i{k}"][r], fx[f"d{k}"][r]
            for dv in np.unique(ref_d):
                if np.sum(ref_d == dv) == 1 and dv != ref_d[-1]:
                    assert i[r][np.argmax(ref_d == dv)] == ref_i[ref_d == dv][0]
            # the k-set can differ only inside the tie group at the boundary
            inner = ref_d < ref_d[-1] - 2e-6
            assert set(ref_i[inner]) <= set(i[r].tolist())


def mmr_scenarios():
    fx = golden("f8_mmr.npz")
    mapping = {int(i): r for r, i in enumerate(fx["ids_all"])}
    for s, name in enumerate(fx["names"]):
        ids = fx[f"s{s}_ids"]
        rows = np.array([mapping.get(int(i), -1) for i in ids], dtype=np.int64)
        yield (str(name), fx["emb"], ids, rows, fx[f"s{s}_scores"], float(fx[f"s{s}_lam"]),
               int(fx[f"s{s}_topk"]), fx[f"s{s}_out"])


def test_f8_mmr_oracle_vs_reference():
    """oracle.mmr_rerank restates main.py:133-169; f8 was made by running it."""
    for name, emb, ids, rows, scores, lam, top_k, expect in mmr_scenarios():
        pos = orc.mmr_rerank(emb, rows, scores, lam, top_k)
        assert [int(ids[p]) for p in pos] == expect.tolist(), name


def test_rank_and_union_oracle():
    s = np.array([0.5, 2.0, 0.5, -1.0, 2.0], np.float32)
    assert orc.rank_by_score(s).tolist() == [1, 4, 0, 2, 3]   # stable on ties
    u = orc.candidate_union([5, 9], np.array([[5, 3, 9, -1], [9, 5, 7, 7]]))
    assert u.tolist() == [3, 5, 7, 9]


def test_f7_reference_service_responses_oracle():
    """F7: the oracle's serving chain (kNN -> union -> [fallback, filters] ->
    fp64 forward -> stable sort -> MMR) on f7_common's caller-side rows gives
    the reference service's ranked hotel ids and similar-item lists."""
    import f7_common
    f = f7_common.load()
    sd = {k: v.double().numpy() for k, v in f.state.items()}
    spec = orc.spec_from_params(f.n_users, f.n_items, f.cat_dims, f.n_num, f.params)
    for req in f.expected["recommendations"]:
        r = f7_common.request_rows(f, req)
        pos = np.asarray(r["pos"], np.int64)
        cand = np.zeros(0, np.int64)
        if len(pos):
            _, nn = orc.cosine_kneighbors(f.emb, f.emb[pos], 11)
            cand = orc.candidate_union(pos, nn)
        if len(cand) < 20:
            cand = np.union1d(cand, np.asarray(r["fallback"], np.int64))
        cand = np.asarray(sorted(set(cand.tolist()) & set(r["allowed"]) - set(r["excluded"])),
                          np.int64)
        got = []
        if len(cand):
            n = len(cand)
            z, _ = orc.forward(sd, spec, np.full(n, r["user_row"], np.int64), cand,
                               f.item_cat[cand], f.item_num[cand])
            order = orc.rank_by_score(z)
            ranked, scores = cand[order], np.asarray(z, np.float32)[order]
            if req["lambda_param"] < 1.0:
                ranked = ranked[orc.mmr_rerank(f.emb, ranked, scores, req["lambda_param"])]
            got = [f.rev[int(x)] for x in ranked]
        assert got == req["ranked_hotels"], (req, got)
    for case in f.expected["similar_items"]:
        row = f.item_map.get(case["item_id"])
        if row is None:
            assert case["status"] == 404
            continue
        _, nn = orc.cosine_kneighbors(f.emb, f.emb[row:row + 1], case["n"] + 1)
        assert [f.rev[int(x)] for x in nn[0, 1:]] == case["ids"], case
