"""Generate the serving golden fixture by running the REFERENCE main.py here.

Run (build container only; /root/reference is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_serving_golden.py

Imports /root/reference/main.py (the FastAPI app object is created, its
lifespan / artifact loading is not run), fills its module-level
``ml_artifacts`` with a synthetic item-embedding table and id mapping, and
records ``rerank_with_mmr`` (main.py:133-169) on several ranked candidate
lists.  Only data is written: tests/golden/f8_mmr.npz.

Scenarios (lambda, n candidates, top_k): all-mapped lists at five lambdas,
unmapped candidates (skipped by the reference), an unmapped first item (its
similarity never counts), duplicate embedding rows (similarity ties), n <
top_k, and n = 1.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def load_main():
    spec = importlib.util.spec_from_file_location("ref_main", os.path.join(REF, "main.py"))
    mod = importlib.util.module_from_spec(spec)
    cwd = os.getcwd()
    os.chdir("/tmp")
    try:
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    return mod


def main():
    ref = load_main()
    rng = np.random.default_rng(8)
    n_rows, d = 500, 16
    emb = rng.standard_normal((n_rows, d)).astype(np.float32)
    emb[1] = emb[0]                 # duplicate rows: equal similarities
    emb[2] = 2.0 * emb[0]
    emb[3] = 0.0                    # zero row: similarity 0 (sklearn normalize)
    ids_all = 1000 + 3 * np.arange(n_rows)          # external hotel ids
    mapping = {int(i): r for r, i in enumerate(ids_all)}
    ref.ml_artifacts['item_embeddings'] = emb
    ref.ml_artifacts['artifacts'] = {'item_id_mapping': mapping}

    out = {"emb": emb, "ids_all": ids_all}
    scen = []

    def add(name, cand_ids, lam, top_k=20):
        scores = np.sort(rng.standard_normal(len(cand_ids)).astype(np.float32))[::-1].copy()
        ranked = list(zip(scores, [int(c) for c in cand_ids]))
        got = ref.rerank_with_mmr(ranked_items_with_scores=ranked, lambda_param=lam, top_k=top_k)
        i = len(scen)
        out[f"s{i}_ids"] = np.asarray(cand_ids, dtype=np.int64)
        out[f"s{i}_scores"] = scores
        out[f"s{i}_lam"] = np.float64(lam)
        out[f"s{i}_topk"] = np.int64(top_k)
        out[f"s{i}_out"] = np.asarray(got, dtype=np.int64)
        scen.append(name)

    base = rng.choice(ids_all, 37, replace=False)
    for lam in (0.0, 0.3, 0.5, 0.7, 0.95):
        add(f"mapped37_l{lam}", base, lam)
    unm = list(rng.choice(ids_all, 120, replace=False))
    for j in range(0, 120, 7):
        unm[j] = 5 + j                               # ids missing from the mapping
    add("unmapped120", unm, 0.5)
    first_unmapped = [7] + list(rng.choice(ids_all, 30, replace=False))
    add("first_unmapped", first_unmapped, 0.6)
    dup = [int(ids_all[0]), int(ids_all[1]), int(ids_all[2]), int(ids_all[3])] + \
        list(rng.choice(ids_all[4:], 56, replace=False))
    add("duplicates", dup, 0.4)
    add("n5", rng.choice(ids_all, 5, replace=False), 0.7)
    add("n1", rng.choice(ids_all, 1, replace=False), 0.7)
    add("top7", rng.choice(ids_all, 50, replace=False), 0.5, top_k=7)
    out["names"] = np.asarray(scen)
    np.savez_compressed(os.path.join(HERE, "f8_mmr.npz"), **out)
    print("wrote f8_mmr.npz:", ", ".join(scen))


if __name__ == "__main__":
    main()
