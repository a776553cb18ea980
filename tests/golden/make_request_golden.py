"""F7: the /recommendations and /similar_items responses of the REFERENCE
service (main.py:170-357) on a synthetic dataset, produced by running the
reference here (build container only; /root/reference is absent on the GPU
box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_request_golden.py

Writes tests/golden/f7_request/: the dataset the service reads (data/*.csv,
as main.py:240-244 loads them), the model artifacts in the formats
train.py:391-396 writes (state_dict .pth, item_embeddings.npy), the
preprocessing artifacts as JSON (mappings, encoders, MinMaxScaler min_/scale_,
numerical columns: the joblib files the reference loads are written to a temp
dir only) and expected.json: the ranked hotel ids per request and the
similar-item lists.  Requests: friends / personal mode, lambda 0.7 / 0.3 /
1.0 (MMR skipped), a user with no reviews (popular-hotel fallback, main.py:
204-207), an unknown user (user row len(map) // 2, main.py:217), a city with
no candidates.  The service's own code runs unchanged: load_artifacts() from
a temp cwd, then the two endpoint functions called directly.
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import tempfile

import numpy as np
import pandas as pd
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_common as gc  # noqa: E402
from make_serving_golden import load_main  # noqa: E402

OUT = os.path.join(HERE, "f7_request")
CITIES = ["Sochi", "Kazan", "Perm"]
CAT_COLS = ["hotel_type", "district"]
NUM_COLS = ["price_rub", "stars", "rating_cleanliness", "rating_service", "rating_location",
            "user_reviews_count", "price_per_star", "cleanliness_vs_service", "location_premium"]
PARAMS = dict(emb_dim=16, hidden_dim=64, n_cross_layers=2, dropout=0.3, n_res_blocks=2)


def make_data(rng):
    n_guests, n_hotels = 70, 90
    hotels = pd.DataFrame({
        "hotel_id": 500 + 7 * np.arange(n_hotels),
        "city": [CITIES[i % 3] for i in range(n_hotels)],
        "price_rub": rng.integers(2000, 20000, n_hotels).astype(float),
        "stars": rng.integers(1, 6, n_hotels).astype(float),
        "hotel_type": rng.choice(["hotel", "hostel", "apart", "resort"], n_hotels),
        "district": rng.choice(["center", "north", "south", "east", "west", "port"], n_hotels),
        "user_reviews_count": rng.integers(0, 500, n_hotels),
    })
    rows = []
    for g in range(n_guests):
        if g in (5, 6):   # guests without reviews
            continue
        for h in rng.choice(n_hotels, rng.integers(3, 12), replace=False):
            r = dict(hotels.iloc[h])
            r["guest_id"] = 100 + g
            r["rating_overall"] = int(rng.integers(1, 11))
            r["rating_cleanliness"] = float(rng.integers(1, 11))
            r["rating_service"] = float(rng.integers(1, 11))
            r["rating_location"] = float(rng.integers(1, 11))
            rows.append(r)
    main = pd.DataFrame(rows).sample(frac=1.0, random_state=3).reset_index(drop=True)
    pairs = set()
    while len(pairs) < 120:
        a, b = rng.integers(0, n_guests, 2)
        if a != b:
            pairs.add((100 + int(min(a, b)), 100 + int(max(a, b))))
    friends = pd.DataFrame(sorted(pairs), columns=["user_id_1", "user_id_2"])
    return main, friends


def main():
    ref = load_main()
    rng = np.random.default_rng(77)
    main_df, friends = make_data(rng)
    # the features main.py:246-252 recreates, for the scaler and encoders
    feat = main_df.rename(columns={"guest_id": "user_id", "hotel_id": "item_id"})
    feat["price_per_star"] = (feat["price_rub"] / feat["stars"]).replace([np.inf, -np.inf], 0).fillna(0)
    feat["cleanliness_vs_service"] = (feat["rating_cleanliness"] / feat["rating_service"]).replace(
        [np.inf, -np.inf], 0).fillna(0)
    feat["location_premium"] = feat["rating_overall"] - feat["rating_location"]
    users = sorted(feat["user_id"].unique().tolist()) + [105, 106]   # 105/106: no reviews
    items = sorted(feat["item_id"].unique().tolist())
    user_map = {int(u): i for i, u in enumerate(users)}
    item_map = {int(h): i for i, h in enumerate(items)}
    encoders = {c: {v: i for i, v in enumerate(sorted(feat[c].unique()))} for c in CAT_COLS}
    from sklearn.preprocessing import MinMaxScaler
    scaler = MinMaxScaler().fit(feat[NUM_COLS])
    cat_dims = {c: len(e) for c, e in encoders.items()}

    torch.manual_seed(42)
    model = ref.DCN_RecSys(len(user_map), len(item_map), cat_dims, len(NUM_COLS), dict(PARAMS))
    gc.perturb_state(model, 43)
    model.eval()

    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(os.path.join(OUT, "data"))
    main_df.to_csv(os.path.join(OUT, "data", "hackathon_augmented_data.csv"), index=False)
    friends.to_csv(os.path.join(OUT, "data", "friendships.csv"), index=False)
    torch.save(model.state_dict(), os.path.join(OUT, "final_dcn_model.pth"))
    np.save(os.path.join(OUT, "item_embeddings.npy"),
            model.item_embedding.weight.detach().cpu().numpy())
    with open(os.path.join(OUT, "artifacts.json"), "w") as f:
        json.dump({"user_id_mapping": {str(k): v for k, v in user_map.items()},
                   "item_id_mapping": {str(k): v for k, v in item_map.items()},
                   "cat_encoders": encoders, "numerical_cols": NUM_COLS,
                   "scaler_min": scaler.min_.tolist(), "scaler_scale": scaler.scale_.tolist(),
                   "model_dims": [len(user_map), len(item_map), cat_dims, len(NUM_COLS)],
                   "best_params": PARAMS}, f, indent=1)

    import joblib
    requests = [(120, "Sochi", "friends", 0.7), (120, "Sochi", "personal", 0.7),
                (131, "Kazan", "friends", 0.3), (131, "Kazan", "personal", 1.0),
                (142, "Perm", "friends", 1.0), (105, "Perm", "personal", 0.7),
                (9999, "Sochi", "friends", 0.7), (157, "Kazan", "friends", 0.5),
                (120, "Atlantis", "friends", 0.7), (163, "Sochi", "personal", 0.0)]
    expected = {"recommendations": [], "similar_items": []}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        shutil.copytree(os.path.join(OUT, "data"), os.path.join(tmp, "data"))
        art = os.path.join(tmp, "artifacts")
        os.makedirs(art)
        joblib.dump({"user_id_mapping": user_map, "item_id_mapping": item_map,
                     "cat_encoders": encoders, "numerical_cols": NUM_COLS, "scaler": scaler},
                    os.path.join(art, "artifacts.gz"))
        joblib.dump((len(user_map), len(item_map), cat_dims, len(NUM_COLS)),
                    os.path.join(art, "model_dims.gz"))
        joblib.dump(dict(PARAMS), os.path.join(art, "best_params.gz"))
        shutil.copy(os.path.join(OUT, "item_embeddings.npy"), art)
        shutil.copy(os.path.join(OUT, "final_dcn_model.pth"), art)
        os.chdir(tmp)
        try:
            ref.load_artifacts()
            for uid, city, mode, lam in requests:
                r = ref.get_recommendations_endpoint(ref.RecommendationRequest(
                    user_id=uid, city=city, type=mode, lambda_param=lam))
                expected["recommendations"].append({
                    "user_id": uid, "city": city, "type": mode, "lambda_param": lam,
                    "ranked_hotels": [int(h["hotel_id"]) for h in r["ranked_hotels"]],
                    "message": r.get("message")})
            for hid, n in [(500, 10), (507, 5), (563, 50), (12345, 10)]:
                try:
                    r = ref.get_similar_items_endpoint(item_id=hid, n=n)
                    expected["similar_items"].append({"item_id": hid, "n": n, "status": 200,
                                                      "ids": [int(x) for x in r["similar_item_ids"]]})
                except ref.HTTPException as e:
                    expected["similar_items"].append({"item_id": hid, "n": n,
                                                      "status": e.status_code, "ids": []})
        finally:
            os.chdir(cwd)
    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(expected, f, indent=1)
    for r in expected["recommendations"]:
        print(r["user_id"], r["city"], r["type"], r["lambda_param"], len(r["ranked_hotels"]),
              r["message"])
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
