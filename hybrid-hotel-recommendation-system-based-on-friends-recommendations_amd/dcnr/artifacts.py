"""The reference's on-disk model artifacts (train.py:391-396 writes them,
main.py:256-270 loads them at API startup):

  final_dcn_model.pth   torch.save(final_model.state_dict())
  item_embeddings.npy   final_model.item_embedding.weight as float32 [n_items, emb_dim]
  model_dims.gz / best_params.gz / artifacts.gz   joblib pickles

``save_artifacts`` writes the first two exactly as train.py:391-394 does;
``load_artifacts`` reads them the way main.py:259-270 uses them, with
loaders that execute nothing from the files (``torch.load(weights_only=True)``,
``np.load(allow_pickle=False)``).  The joblib files are pickles: their
values (``model_dims = (n_users, n_items, cat_dims, n_num_features)`` and
``best_params``) are passed in by the caller, who decides whether to trust
them.  The state_dict is interchangeable both ways with the reference's
``DCN_RecSys`` (same keys, shapes, dtypes).
"""
from __future__ import annotations

import os
from typing import Any, Dict, Tuple

import numpy as np
import torch

from .knn import NearestNeighbors
from .model import DCN_RecSys

MODEL_FILE = "final_dcn_model.pth"
EMB_FILE = "item_embeddings.npy"


def save_artifacts(model: DCN_RecSys, artifacts_dir: str) -> None:
    """train.py:391-394: the state_dict and the item-embedding table."""
    os.makedirs(artifacts_dir, exist_ok=True)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save(sd, os.path.join(artifacts_dir, MODEL_FILE))
    emb = model.item_embedding.weight.detach().cpu().numpy()
    np.save(os.path.join(artifacts_dir, EMB_FILE), emb)


def load_artifacts(artifacts_dir: str, model_dims: Tuple[int, int, Dict[str, int], int],
                   best_params: Dict[str, Any], device="cuda", precision="fp32",
                   n_neighbors: int = 16) -> Tuple[DCN_RecSys, np.ndarray, NearestNeighbors]:
    """main.py:259-270: build DCN_RecSys(*model_dims, best_params), load the
    state_dict, move to the device in eval mode, load the item embeddings and
    fit the cosine index on them.  Returns (model, item_embeddings, index)."""
    n_users, n_items, cat_dims, n_num_features = model_dims
    model = DCN_RecSys(n_users, n_items, cat_dims, n_num_features, best_params,
                       precision=precision)
    sd = torch.load(os.path.join(artifacts_dir, MODEL_FILE), map_location="cpu",
                    weights_only=True)
    model.load_state_dict(sd)
    model.to(device)
    model.eval()
    emb = np.load(os.path.join(artifacts_dir, EMB_FILE), allow_pickle=False)
    index = NearestNeighbors(n_neighbors=n_neighbors, metric="cosine", algorithm="brute",
                             device=device).fit(emb)
    return model, emb, index
