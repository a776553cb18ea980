"""F9: the reference's on-disk model artifacts, written by the REFERENCE code
in this container (build container only; /root/reference is absent on the
GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_artifacts_golden.py

Builds F1's model with the reference's ``DCN_RecSys`` (train.py:125-153;
golden_common.build: seed 42 + perturb_state) and saves what train.py:391-394
saves -- ``torch.save(model.state_dict())`` and the item-embedding table
with ``np.save`` -- into tests/golden/f9_artifacts/.  F1's logits
(f1_cfg1_eval.npz) are those of this model on F1's inputs, so loading the
files into our model and scoring F1's inputs on the GPU must reproduce them.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_common as gc  # noqa: E402
from make_golden import load_reference  # noqa: E402


def main():
    ref = load_reference()
    m = gc.build(ref.DCN_RecSys, gc.CFG1).eval()
    out = os.path.join(HERE, "f9_artifacts")
    os.makedirs(out, exist_ok=True)
    torch.save(m.state_dict(), os.path.join(out, "final_dcn_model.pth"))
    np.save(os.path.join(out, "item_embeddings.npy"), m.item_embedding.weight.detach().cpu().numpy())
    print("wrote", sorted(os.listdir(out)))


if __name__ == "__main__":
    main()
