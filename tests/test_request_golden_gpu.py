"""F7: the reference service's /recommendations and
/similar_items responses (main.py:170-357, run here by
tests/golden/make_request_golden.py on a synthetic dataset) reproduced by
``dcnr.RankingPipeline`` on the GPU.

The test is the service's caller: tests/f7_common.py restates main.py's
host-side pandas steps and hands the device path what main.py hands the
model and the index (hotel rows, the user row, the filters).  Everything from
candidate generation to the MMR order runs in libdcnr (top-k, candidate
union, ranking batch, eval forward, stable sort, MMR).  The ranked hotel ids
must equal the reference's response exactly (fp32 model; the reference ran
on the CPU).  tests/test_oracle_golden.py checks the oracle on the same
fixture.
"""
import pytest
import torch

import f7_common

pytestmark = pytest.mark.gpu


def _pipe(f, dev):
    import dcnr
    m = dcnr.DCN_RecSys(f.n_users, f.n_items, f.cat_dims, f.n_num, dict(f.params),
                        precision="fp32")
    m.load_state_dict(f.state)
    m = m.to(dev).eval()
    return dcnr.RankingPipeline(m, f.item_cat, f.item_num,
                                item_embeddings=torch.from_numpy(f.emb).to(dev))


def test_f7_recommendations_match_reference(dev):
    f = f7_common.load()
    pipe = _pipe(f, dev)
    n_mmr = 0
    for req in f.expected["recommendations"]:
        r = f7_common.request_rows(f, req)
        rows, _ = pipe.recommend(r["user_row"], r["pos"], lambda_param=req["lambda_param"],
                                 allowed=r["allowed"], excluded=r["excluded"],
                                 fallback=r["fallback"])
        got = [f.rev[x] for x in rows.tolist()]
        assert got == req["ranked_hotels"], (req, got)
        n_mmr += req["lambda_param"] < 1.0 and len(got) > 1
    assert n_mmr >= 5 and any(len(r["ranked_hotels"]) == 0 for r in f.expected["recommendations"])


def test_f7_similar_items_match_reference(dev):
    f = f7_common.load()
    pipe = _pipe(f, dev)
    for case in f.expected["similar_items"]:
        row = f.item_map.get(case["item_id"])
        if row is None:   # main.py:297-298: HTTP 404
            assert case["status"] == 404
            continue
        got = [f.rev[x] for x in pipe.similar_items(row, case["n"]).tolist()]
        assert case["status"] == 200 and got == case["ids"], (case, got)
