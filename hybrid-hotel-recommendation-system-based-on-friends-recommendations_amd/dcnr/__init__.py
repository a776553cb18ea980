"""dcnr -- MI355X-native (gfx950 HIP) DCN-R ranking path.

Drop-in surfaces of the reference (Krist-Marrakesh/Hybrid-Hotel-Recommendation-
System-Based-on-Friends-Recommendations):

  DCN_RecSys, CrossLayer, ResBlock   train.py:90-170 / main.py:61-127
  BCEWithLogitsLoss                  train.py:206
  AdamW, Adam                        train.py:201-204
  NearestNeighbors (cosine, brute)   main.py:268-270
  FusedTrainer                       the train.py:219-226 inner-loop step
  DeviceLoader                       TensorDataset + DataLoader (train.py:195-196)
  serving.rerank_with_mmr            main.py:133-169
  serving.RankingPipeline            the /recommendations + /similar_items core
                                     (main.py:196-230, 294-332)
  artifacts.save_artifacts /         final_dcn_model.pth + item_embeddings.npy
  artifacts.load_artifacts           (train.py:391-394, main.py:256-270)

All compute runs in libdcnr.so (C ABI: include/dcnr.h) on the HIP device.
"""
from .model import CrossLayer, DCN_RecSys, ResBlock  # noqa: F401
from .ops import Adam, AdamW, BCEWithLogitsLoss, bce_with_logits  # noqa: F401
from .knn import NearestNeighbors, ShardedNearestNeighbors  # noqa: F401
from .train import FusedTrainer  # noqa: F401
from . import serving  # noqa: F401
from .data import DeviceLoader  # noqa: F401
from .serving import RankingPipeline, rerank_with_mmr  # noqa: F401
from . import artifacts  # noqa: F401

__version__ = "0.1.0"
