"""The /recommendations and /similar_items scoring core on libdcnr.

Mirrors the reference's serving functions (main.py) with their device work in
HIP kernels (serving.hip, knn.hip, the DCN-R forward):

  rerank_with_mmr(ranked_items_with_scores, lambda_param, top_k=20)
      main.py:133-169, same signature; reads ``ml_artifacts['item_embeddings']``
      and ``ml_artifacts['artifacts']['item_id_mapping']`` like the reference
      (this module's ``ml_artifacts`` dict), greedy MMR in one launch
      (dcnr_mmr_rerank).
  RankingPipeline
      the device-resident request path: cosine neighbours of the positive
      hotels for ALL positives in one batched top-k (main.py:196-203 calls
      kneighbors once per hotel), the candidate union (dcnr_candidate_union),
      the ranking batch of preprocess_for_ranking (main.py:215-230) gathered
      from per-item feature tables (dcnr_ranking_batch), the eval-mode DCN-R
      forward (main.py:319-322), the stable descending sort (main.py:325,
      dcnr_rank_by_score) and MMR (main.py:327-332).

Everything works on internal row indices (the reference's ``item_id_mapping``
values); mapping external ids stays with the caller, as in main.py.  The
pandas filters of _generate_candidates (city, negative reviews, popular-hotel
fill-up, main.py:204-212) are host set operations and take ``allowed`` /
``excluded`` row sets here.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .knn import NearestNeighbors

ml_artifacts: Dict[str, Any] = {}

SV_MAX = 4096   # csrc/serving.hip: candidates per union / rank / MMR call

def _dev_table(emb, device):
    """(table fp32 [n, d] on device, inverse row norms [n]) cached per source array."""
    cache = ml_artifacts.setdefault('_dcnr_tables', {})
    key = id(emb)
    hit = cache.get(key)
    if hit is not None and hit[0] is emb:
        return hit[1], hit[2]
    t = torch.as_tensor(np.asarray(emb, dtype=np.float32) if not torch.is_tensor(emb) else emb)
    t = t.to(device, torch.float32).contiguous()
    inv = row_inv_norms(t)
    cache[key] = (emb, t, inv)
    return t, inv


def row_inv_norms(t: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    inv = torch.empty(t.shape[0], dtype=torch.float32, device=t.device)
    _lib.check(lib.dcnr_row_inv_norms(t.data_ptr(), t.shape[0], t.shape[1], inv.data_ptr(),
                                      _lib.stream_ptr(t.device)), "dcnr_row_inv_norms")
    return inv


def mmr_positions(table: torch.Tensor, inv: torch.Tensor, rows: torch.Tensor,
                  scores: torch.Tensor, lambda_param: float, top_k: int = 20) -> torch.Tensor:
    """Device MMR over candidates in ranked order: returns int64 positions
    (into the ranked list) of the re-ranked items (dcnr_mmr_rerank).  At most
    SV_MAX candidates (one workgroup's LDS holds every candidate's running
    max-similarity); more raise ValueError."""
    lib = _lib.load()
    dev = table.device
    n = rows.numel()
    if n > SV_MAX:
        raise ValueError(f"mmr_positions: {n} candidates exceed the device MMR's {SV_MAX}")
    out = torch.empty(max(1, top_k), dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    if n == 0:
        return out[:0]
    rows = rows.to(dev, torch.int64).contiguous()
    scores = scores.to(dev, torch.float32).contiguous()
    _lib.check(lib.dcnr_mmr_rerank(table.data_ptr(), inv.data_ptr(), table.shape[1],
                                   rows.data_ptr(), scores.data_ptr(), n, float(lambda_param),
                                   int(top_k), out.data_ptr(), cnt.data_ptr(),
                                   _lib.stream_ptr(dev)), "dcnr_mmr_rerank")
    return out[:int(cnt.item())]


def rerank_with_mmr(ranked_items_with_scores: List[Tuple[float, int]], lambda_param: float,
                    top_k: int = 20) -> List[int]:
    """main.py:133-169: greedy Maximal Marginal Relevance over (score, item_id)
    pairs given in ranked order; returns the re-ranked item ids."""
    if not ranked_items_with_scores:
        return []
    emb = ml_artifacts['item_embeddings']
    mapping = ml_artifacts['artifacts']['item_id_mapping']
    device = ml_artifacts.get('device', torch.device('cuda'))
    if isinstance(device, str):
        device = torch.device(device)
    if device.type != 'cuda':
        raise RuntimeError("dcnr.serving runs on the HIP device only")
    table, inv = _dev_table(emb, device)
    ids = [item_id for _, item_id in ranked_items_with_scores]
    rows = torch.tensor([mapping.get(i, -1) if mapping.get(i) is not None else -1 for i in ids],
                        dtype=torch.int64)
    scores = torch.tensor(np.asarray([s for s, _ in ranked_items_with_scores], dtype=np.float32))
    pos = mmr_positions(table, inv, rows, scores, lambda_param, top_k).cpu().tolist()
    return [ids[p] for p in pos]


class RankingPipeline:
    """Device-resident request path of /recommendations and /similar_items.

    model      dcnr.DCN_RecSys (eval mode is set here), on the HIP device
    item_embeddings  [n_items, d] (the exported item_embedding weights,
               train.py:393-394); default: the model's own item table
    item_cat   int64 [n_items, n_cat]: each hotel's encoded categorical codes
    item_num   fp32 [n_items, n_num]: each hotel's scaled numeric features
    """

    def __init__(self, model, item_cat, item_num, item_embeddings=None, n_neighbors: int = 11):
        dev = model.final_linear.weight.device
        if dev.type != 'cuda':
            raise RuntimeError("RankingPipeline runs on the HIP device only")
        self.model = model.eval()
        self.device = dev
        emb = model.item_embedding.weight.detach() if item_embeddings is None else item_embeddings
        self.index = NearestNeighbors(n_neighbors=n_neighbors, metric='cosine',
                                      algorithm='brute', device=dev).fit(emb)
        self.item_cat = torch.as_tensor(item_cat).to(dev, torch.int64).contiguous()
        self.item_num = torch.as_tensor(item_num).to(dev, torch.float32).contiguous()
        self.n_items = self.item_cat.shape[0]
        self.n_neighbors = n_neighbors
        if self.item_num.shape[0] != self.n_items:
            raise ValueError("item_cat and item_num must have one row per item")

    # ---------------------------------------------------------- /similar_items
    def similar_items(self, item_row: int, n: int = 10) -> torch.Tensor:
        """main.py:294-303: the n nearest hotels, the hotel itself dropped
        (kneighbors(n_neighbors=n+1)[1:])."""
        q = self.index._table[int(item_row)].reshape(1, -1)
        _, idx = self.index.kneighbors_device(q, n + 1)
        return idx[0, 1:]

    # ------------------------------------------------------- /recommendations
    def candidates(self, positive_rows) -> torch.Tensor:
        """_generate_candidates' union (main.py:196-203): the positive hotels
        and their n_neighbors-1 nearest neighbours, distinct rows ascending."""
        lib = _lib.load()
        pos = torch.as_tensor(positive_rows, dtype=torch.int64).reshape(-1).to(self.device)
        Q = pos.numel()
        if Q == 0:
            return pos
        k = self.n_neighbors
        _, idx = self.index.kneighbors_device(self.index._table[pos], k)
        qc = max(1, SV_MAX // k)     # the union kernel's one-workgroup capacity
        outs = []
        for q0 in range(0, Q, qc):   # > SV_MAX entries: per-chunk unions, then merged
            p_, i_ = pos[q0:q0 + qc].contiguous(), idx[q0:q0 + qc].contiguous()
            out = torch.empty(p_.numel() * k, dtype=torch.int64, device=self.device)
            cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
            _lib.check(lib.dcnr_candidate_union(p_.data_ptr(), p_.numel(), i_.data_ptr(), k,
                                                out.data_ptr(), cnt.data_ptr(),
                                                _lib.stream_ptr(self.device)),
                       "dcnr_candidate_union")
            outs.append(out[:int(cnt.item())])
        if len(outs) == 1:
            return outs[0]
        return torch.unique(torch.cat(outs))   # ascending distinct rows, as one call gives

    def ranking_batch(self, user_row: int, item_rows: torch.Tensor):
        """preprocess_for_ranking (main.py:215-230) on the device."""
        lib = _lib.load()
        item_rows = item_rows.to(self.device, torch.int64).contiguous()
        n = item_rows.numel()
        K, F = self.item_cat.shape[1], self.item_num.shape[1]
        u = torch.empty(n, dtype=torch.int64, device=self.device)
        i = torch.empty(n, dtype=torch.int64, device=self.device)
        c = torch.empty((n, K), dtype=torch.int64, device=self.device)
        x = torch.empty((n, F), dtype=torch.float32, device=self.device)
        _lib.check(lib.dcnr_ranking_batch(item_rows.data_ptr(), n, int(user_row),
                                          self.item_cat.data_ptr() if K else None, K,
                                          self.item_num.data_ptr() if F else None, F,
                                          self.n_items, u.data_ptr(), i.data_ptr(),
                                          c.data_ptr() if K else None,
                                          x.data_ptr() if F else None,
                                          _lib.stream_ptr(self.device)), "dcnr_ranking_batch")
        return u, i, c, x

    @torch.no_grad()
    def score(self, user_row: int, item_rows: torch.Tensor) -> torch.Tensor:
        """Eval-mode DCN-R logits of (user, hotel) pairs (main.py:319-322)."""
        if item_rows.numel() == 0:
            return torch.empty(0, dtype=torch.float32, device=self.device)
        return self.model(*self.ranking_batch(user_row, item_rows)).reshape(-1)

    def rank(self, scores: torch.Tensor) -> torch.Tensor:
        """Positions in descending score order, ties by position (main.py:325).
        Above SV_MAX candidates (the LDS sort's capacity) a stable device sort
        of -score gives the same order."""
        lib = _lib.load()
        n = scores.numel()
        if n > SV_MAX:
            return torch.sort(-scores.to(self.device, torch.float32), stable=True).indices
        order = torch.empty(n, dtype=torch.int64, device=self.device)
        if n:
            s = scores.to(torch.float32).contiguous()
            _lib.check(lib.dcnr_rank_by_score(s.data_ptr(), n, order.data_ptr(),
                                              _lib.stream_ptr(self.device)), "dcnr_rank_by_score")
        return order

    @torch.no_grad()
    def recommend(self, user_row: int, positive_rows, lambda_param: float = 1.0,
                  top_k: int = 20, allowed: Optional[Iterable[int]] = None,
                  excluded: Optional[Iterable[int]] = None,
                  fallback: Optional[Iterable[int]] = None, min_candidates: int = 20):
        """The scoring core of /recommendations (main.py:309-332) on hotel rows:
        candidates -> [fallback] -> [filters] -> ranking batch -> logits ->
        sort -> MMR when lambda_param < 1.  ``fallback`` (the city's most
        reviewed hotels) joins the candidates when fewer than
        ``min_candidates`` were found (main.py:204-207).  Returns (ranked
        rows, their logits) on the device."""
        cand = self.candidates(positive_rows)
        if fallback is not None and cand.numel() < min_candidates:
            extra = torch.as_tensor(list(fallback), dtype=torch.int64).to(self.device)
            cand = torch.unique(torch.cat([cand, extra]))
        if allowed is not None or excluded is not None:   # host set filters (main.py:210-212)
            keep = set(cand.tolist())
            if allowed is not None:
                keep &= set(int(a) for a in allowed)
            if excluded is not None:
                keep -= set(int(e) for e in excluded)
            cand = torch.tensor(sorted(keep), dtype=torch.int64, device=self.device)
        if cand.numel() == 0:   # "No suitable candidates found." (main.py:311-312)
            return cand, torch.empty(0, dtype=torch.float32, device=self.device)
        scores = self.score(user_row, cand)
        order = self.rank(scores)
        ranked, rscores = cand[order], scores[order]
        if lambda_param < 1.0 and ranked.numel():
            pos = mmr_positions(self.index._table, self.index._inv, ranked, rscores,
                                lambda_param, top_k)
            return ranked[pos], rscores[pos]
        return ranked, rscores
