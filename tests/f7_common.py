"""F7 (tests/golden/f7_request, written by make_request_golden.py running the
reference service): the service's caller-side steps restated, shared by the
GPU test (libdcnr does the device path) and the CPU test (the oracle does).

``load()`` reads the dataset and artifacts as main.py's load_artifacts does
(main.py:240-266; JSON instead of joblib, the state_dict weights-only) and
builds each hotel's ranking features from its first main_df row, encoded and
scaled as preprocess_for_ranking does (main.py:215-230).  ``request_rows()``
restates _generate_candidates' host part (main.py:170-212): the positives and
negatives of the user (personal) or the friends (friends mode), the city's
most-reviewed hotels for the < 20-candidate fallback, the city's hotels, the
user row (unknown users -> len(map) // 2, main.py:217) -- as hotel rows.
"""
import json
import os

import numpy as np
import pandas as pd
import torch

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "f7_request")


class F7:
    pass


def load():
    f = F7()
    art = json.load(open(os.path.join(DIR, "artifacts.json")))
    main_df = pd.read_csv(os.path.join(DIR, "data", "hackathon_augmented_data.csv"))
    main_df.rename(columns={"guest_id": "user_id", "hotel_id": "item_id"}, inplace=True)
    main_df["price_per_star"] = (main_df["price_rub"] / main_df["stars"]).replace(
        [np.inf, -np.inf], 0).fillna(0)
    main_df["cleanliness_vs_service"] = (main_df["rating_cleanliness"] /
                                         main_df["rating_service"]).replace([np.inf, -np.inf], 0).fillna(0)
    main_df["location_premium"] = main_df["rating_overall"] - main_df["rating_location"]
    f.main_df = main_df
    f.friends = pd.read_csv(os.path.join(DIR, "data", "friendships.csv"))
    f.user_map = {int(k): v for k, v in art["user_id_mapping"].items()}
    f.item_map = {int(k): v for k, v in art["item_id_mapping"].items()}
    f.rev = {v: k for k, v in f.item_map.items()}
    f.n_users, f.n_items, f.cat_dims, f.n_num = art["model_dims"]
    f.params = dict(art["best_params"])
    f.state = torch.load(os.path.join(DIR, "final_dcn_model.pth"), weights_only=True)
    f.emb = np.load(os.path.join(DIR, "item_embeddings.npy"))
    first = main_df.drop_duplicates(subset=["item_id"]).set_index("item_id")
    f.item_cat = np.zeros((f.n_items, len(art["cat_encoders"])), np.int64)
    f.item_num = np.zeros((f.n_items, f.n_num), np.float32)
    mn, sc = np.array(art["scaler_min"]), np.array(art["scaler_scale"])
    for h, r in f.item_map.items():
        row = first.loc[h]
        f.item_cat[r] = [enc.get(str(row[c]), 0) for c, enc in art["cat_encoders"].items()]
        x = row[art["numerical_cols"]].to_numpy(np.float64)
        f.item_num[r] = (x * sc + mn).astype(np.float32)   # MinMaxScaler.transform, then fp32
    f.expected = json.load(open(os.path.join(DIR, "expected.json")))
    return f


def _friends_of(friends, uid):   # main.py:170-176
    return set(friends[friends["user_id_1"] == uid]["user_id_2"].tolist() +
               friends[friends["user_id_2"] == uid]["user_id_1"].tolist())


def request_rows(f, req):
    uid, city, mode = req["user_id"], req["city"], req["type"]
    df = f.main_df
    if mode == "friends":
        src = _friends_of(f.friends, uid)
        reviews = df[df["user_id"].isin(src)] if src else pd.DataFrame()
    else:
        reviews = df[df["user_id"] == uid]
    pos, neg = [], set()
    if not reviews.empty:
        pos = reviews[reviews["rating_overall"] >= 8]["item_id"].unique().tolist()
        neg = set(reviews[reviews["rating_overall"] <= 4]["item_id"].unique())
    popular = df[df["city"] == city].sort_values(by="user_reviews_count",
                                                 ascending=False).head(100)["item_id"].tolist()
    city_hotels = set(df[df["city"] == city]["item_id"].unique())
    return dict(user_row=f.user_map.get(uid, len(f.user_map) // 2),
                pos=[f.item_map[h] for h in pos],
                allowed=sorted(f.item_map[h] for h in city_hotels),
                excluded=sorted(f.item_map[h] for h in neg),
                fallback=[f.item_map[h] for h in popular])
