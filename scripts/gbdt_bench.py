"""GBDT on one MI355X: histogram kernel throughput and end-to-end boosting time.

Synthetic HIGGS-shaped data (rows x 28 float features, binary label), xgboost defaults
(depth 6, eta 0.3, max_bin 256). Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from ray_community_amd import ops
from ray_community_amd.train.gbdt import DMatrix, train

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2_000_000)
ap.add_argument("--features", type=int, default=28)
ap.add_argument("--rounds", type=int, default=50)
ap.add_argument("--hist-only", action="store_true")
a = ap.parse_args()

rng = np.random.default_rng(0)
X = rng.normal(size=(a.rows, a.features)).astype(np.float32)
w = rng.normal(size=a.features).astype(np.float32)
y = ((X @ w + 0.5 * np.sin(3 * X[:, 0]) * X[:, 1]) > 0).astype(np.float32)
dev = "cuda"

# histogram kernel alone: all rows in L nodes
ld = (a.rows + 3) // 4 * 4
bins = torch.randint(0, 256, (a.features, ld), dtype=torch.uint8, device=dev)
gh = torch.randn(ld, 2, device=dev)
for L in (1, 8, 32):
    node = torch.randint(0, L, (ld,), dtype=torch.int32, device=dev)
    out = torch.zeros(L, a.features, 256, 2, device=dev)
    for _ in range(3):
        ops.gbdt_histogram(bins, node, gh, L, out=out)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        ops.gbdt_histogram(bins, node, gh, L, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    byts = a.features * ld + ld * (4 + 8)
    print(json.dumps({"metric": "gbdt_hist", "nodes": L, "rows": a.rows, "features": a.features,
                      "us": round(dt * 1e6, 1), "GB/s": round(byts / dt / 1e9, 1),
                      "Grow_feat_per_s": round(a.rows * a.features / dt / 1e9, 2)}), flush=True)

if a.hist_only:
    sys.exit(0)
d = DMatrix(X, y, device=dev)
train({"objective": "binary:logistic"}, d, 2)  # warm-up (sketch + binning cached on d)
torch.cuda.synchronize()
res = {}
t = time.perf_counter()
b = train({"objective": "binary:logistic", "eval_metric": ["logloss", "error"]}, d, a.rounds,
          evals=[(d, "train")], evals_result=res)
torch.cuda.synchronize()
dt = time.perf_counter() - t
print(json.dumps({"metric": "gbdt_train", "rows": a.rows, "features": a.features, "rounds": a.rounds,
                  "max_depth": 6, "s_total": round(dt, 2), "ms_per_round": round(dt / a.rounds * 1e3, 1),
                  "train_error": round(res["train"]["error"][-1], 4)}), flush=True)
