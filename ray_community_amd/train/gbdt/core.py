"""Data-parallel histogram gradient-boosted decision trees (the engine behind ``XGBoostTrainer`` /
``LightGBMTrainer``).

The reference's GBDT trainers orchestrate the xgboost / lightgbm libraries
(``python/ray/train/xgboost/xgboost_trainer.py:18-67``: every worker turns its dataset shard into a
DMatrix and ``xgboost.train`` runs inside a rabit ``CommunicatorContext``;
``python/ray/train/lightgbm/lightgbm_trainer.py``). Neither library exists on this image, and the
point of a native trainer is that the boosting itself runs on the MI355X, so this module implements
the algorithm those libraries use for distributed training:

* **quantile sketch** -- every worker samples its shard, the per-feature quantile points of all
  workers are all-gathered and merged into <= 254 cut points per feature (bin 255 = missing);
* **quantised matrix** -- feature-major uint8 ``[F, rows]`` resident in HBM for the whole run;
* **histograms** -- per round and tree level, (grad, hess[, count]) histograms of the nodes being
  expanded come from ``ops.gbdt_histogram`` (``ops/csrc/gbdt.hip``: LDS-private per-workgroup
  histograms) and are summed across workers with one all-reduce (RCCL on GPU, gloo on CPU); the
  sibling of the smaller child is parent - child (histogram subtraction);
* **split finding** -- vectorised over nodes x features x bins x {missing left, missing right}
  with the second-order gain ``T(G_L)^2/(H_L+lambda) + T(G_R)^2/(H_R+lambda) - T(G)^2/(H+lambda)``
  (``T`` = L1 soft threshold), ``min_child_weight`` / ``min_data_in_leaf`` / ``gamma`` constraints,
  learned default directions for missing values;
* **growth policies** -- ``depthwise`` (xgboost default, level by level up to ``max_depth``) and
  ``lossguide`` (lightgbm default, best-gain leaf first up to ``max_leaves`` / ``num_leaves``);
* row subsampling and per-tree column subsampling with a shared seed (all workers agree on the
  column mask; row masks are per-worker streams).

Every worker ends with the identical model (split decisions only depend on all-reduced
statistics), so rank 0 can checkpoint it. Objectives: squared error, logistic, softmax;
metrics: rmse / mae / (binary, multi) logloss / error, also under the lightgbm names.
"""
from __future__ import annotations

import json
import math
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

MISSING_BIN = 255
NBINS = 256

# ----------------------------------------------------------------------------- distributed helpers


def _world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _comm_device(t: torch.Tensor) -> torch.device:
    if _world() > 1 and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return t.device


def allreduce_sum(t: torch.Tensor) -> torch.Tensor:
    """In-place sum over workers (no-op at world 1)."""
    if _world() == 1:
        return t
    dev = _comm_device(t)
    if dev != t.device:
        x = t.to(dev)
        dist.all_reduce(x)
        t.copy_(x.to(t.device))
    else:
        dist.all_reduce(t)
    return t


def allgather_cat(t: torch.Tensor) -> torch.Tensor:
    """Concatenate equal-shaped tensors of all workers along a new leading dim."""
    if _world() == 1:
        return t.unsqueeze(0)
    dev = _comm_device(t)
    x = t.to(dev).contiguous()
    out = [torch.empty_like(x) for _ in range(_world())]
    dist.all_gather(out, x)
    return torch.stack(out).to(t.device)


# ----------------------------------------------------------------------------- parameters

_ALIASES = {
    "learning_rate": "eta", "shrinkage_rate": "eta",
    "reg_lambda": "lambda", "lambda_l2": "lambda", "l2_regularization": "lambda",
    "reg_alpha": "alpha", "lambda_l1": "alpha",
    "min_split_loss": "gamma", "min_gain_to_split": "gamma",
    "min_sum_hessian_in_leaf": "min_child_weight", "min_hessian": "min_child_weight",
    "min_data_in_leaf": "min_data_in_leaf", "min_child_samples": "min_data_in_leaf",
    "bagging_fraction": "subsample", "feature_fraction": "colsample_bytree",
    "num_leaves": "max_leaves", "random_state": "seed", "random_seed": "seed",
    "metric": "eval_metric", "num_class": "num_class", "nthread": None, "n_jobs": None,
    "tree_method": None, "device": None, "verbosity": None, "verbose": None, "num_threads": None,
}

_XGB_DEFAULTS = dict(eta=0.3, max_depth=6, grow_policy="depthwise", max_leaves=0, **{"lambda": 1.0}, alpha=0.0,
                     gamma=0.0, min_child_weight=1.0, min_data_in_leaf=0, subsample=1.0, colsample_bytree=1.0,
                     max_bin=256, seed=0, objective="reg:squarederror", num_class=1, base_score=None,
                     eval_metric=None, hist_precision="auto")
_LGB_DEFAULTS = dict(_XGB_DEFAULTS, eta=0.1, max_depth=-1, grow_policy="lossguide", max_leaves=31,
                     **{"lambda": 0.0}, min_child_weight=1e-3, min_data_in_leaf=20, max_bin=255,
                     objective="regression")

_OBJECTIVES = {
    "reg:squarederror": "squared", "reg:linear": "squared", "regression": "squared", "regression_l2": "squared",
    "l2": "squared", "mse": "squared", "mean_squared_error": "squared",
    "binary:logistic": "logistic", "binary": "logistic", "binary:logitraw": "logistic_raw",
    "multi:softprob": "softprob", "multiclass": "softprob", "softmax": "softprob",
    "multi:softmax": "softmax",
}

_DEFAULT_METRIC = {"squared": "rmse", "logistic": "logloss", "logistic_raw": "logloss", "softprob": "mlogloss",
                   "softmax": "mlogloss"}
_LGB_DEFAULT_METRIC = {"squared": "l2", "logistic": "binary_logloss", "logistic_raw": "binary_logloss",
                       "softprob": "multi_logloss", "softmax": "multi_logloss"}


def normalize_params(params: Optional[Dict[str, Any]], flavor: str = "xgboost") -> Dict[str, Any]:
    """xgboost / lightgbm parameter names -> one canonical dict (defaults of that library)."""
    out = dict(_LGB_DEFAULTS if flavor == "lightgbm" else _XGB_DEFAULTS)
    for k, v in (params or {}).items():
        k2 = _ALIASES.get(k, k)
        if k2 is None:
            continue
        out[k2] = v
    obj = out["objective"]
    if obj not in _OBJECTIVES:
        raise ValueError(f"Unsupported objective {obj!r}; supported: {sorted(_OBJECTIVES)}")
    out["_obj"] = _OBJECTIVES[obj]
    if out["_obj"] in ("softprob", "softmax") and int(out.get("num_class") or 0) < 2:
        raise ValueError(f"objective {obj!r} needs num_class >= 2")
    if out["_obj"] not in ("softprob", "softmax"):
        out["num_class"] = 1
    if flavor == "lightgbm" and int(out["max_depth"]) <= 0:
        out["max_depth"] = 0  # unlimited
    if out["grow_policy"] == "lossguide" and int(out["max_leaves"]) <= 0:
        out["max_leaves"] = 31
    em = out.get("eval_metric")
    if em is None or em == "" or em == []:
        em = (_LGB_DEFAULT_METRIC if flavor == "lightgbm" else _DEFAULT_METRIC)[out["_obj"]]
    out["eval_metric"] = [em] if isinstance(em, str) else list(em)
    out["max_bin"] = int(max(2, min(int(out["max_bin"]), 255)))
    out["_flavor"] = flavor
    return out


# ----------------------------------------------------------------------------- data


def _to_tensor(x, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.float32)
    try:
        import pandas as pd

        if isinstance(x, (pd.DataFrame, pd.Series)):
            x = x.to_numpy(dtype=np.float32, na_value=np.nan)
    except ImportError:  # pragma: no cover
        pass
    return torch.as_tensor(np.asarray(x, dtype=np.float32), device=device)


class DMatrix:
    """Features (+ label) of one worker's shard, xgboost.DMatrix-like. ``data``: numpy / pandas /
    torch [N, F] (NaN = missing); quantised lazily against the booster's cut points."""

    def __init__(self, data, label=None, *, feature_names: Optional[List[str]] = None, weight=None,
                 device: Optional[str] = None):
        dev = torch.device(device) if device is not None else torch.device("cpu")
        try:
            import pandas as pd

            if isinstance(data, pd.DataFrame) and feature_names is None:
                feature_names = [str(c) for c in data.columns]
        except ImportError:  # pragma: no cover
            pass
        self.X = _to_tensor(data, dev)
        if self.X.dim() == 1:
            self.X = self.X[:, None]
        self.y = None if label is None else _to_tensor(label, dev).reshape(-1)
        self.w = None if weight is None else _to_tensor(weight, dev).reshape(-1)
        self.feature_names = feature_names or [f"f{i}" for i in range(self.X.shape[1])]
        self._binned: Optional[Tuple[int, torch.Tensor]] = None

    @property
    def device(self):
        return self.X.device

    def num_row(self) -> int:
        return int(self.X.shape[0])

    def num_col(self) -> int:
        return int(self.X.shape[1])

    def binned(self, cuts: List[torch.Tensor]) -> torch.Tensor:
        """uint8 [F, ld] feature-major quantised copy (ld = rows padded to a multiple of 4)."""
        key = id(cuts)
        if self._binned is not None and self._binned[0] == key:
            return self._binned[1]
        N, F = self.X.shape
        ld = (N + 3) // 4 * 4
        out = torch.full((F, ld), MISSING_BIN, dtype=torch.uint8, device=self.device)
        for f in range(F):
            col = self.X[:, f]
            b = torch.searchsorted(cuts[f], col.contiguous(), right=True)
            b = torch.where(torch.isnan(col), torch.full_like(b, MISSING_BIN), b)
            out[f, :N] = b.to(torch.uint8)
        self._binned = (key, out)
        return out


def sketch_cuts(X: torch.Tensor, max_bin: int, seed: int = 0, sample: int = 200_000) -> List[torch.Tensor]:
    """Per-feature cut points from a distributed quantile sketch: every worker's local quantile
    points (at 4 x max_bin levels, NaNs ignored) are all-gathered and merged; features with few
    distinct values get one bin per value."""
    N, F = X.shape
    g = torch.Generator(device="cpu").manual_seed(seed + 7919 * (dist.get_rank() if _world() > 1 else 0))
    Xs = X if N <= sample else X[torch.randperm(N, generator=g)[:sample].to(X.device)]
    Xs = Xs.float()
    Q = 4 * max_bin + 1
    qs = torch.linspace(0, 1, Q, device=X.device)
    pts = torch.full((F, Q), float("nan"), device=X.device)
    for f in range(F):
        col = Xs[:, f]
        col = col[~torch.isnan(col)]
        if col.numel():
            pts[f] = torch.quantile(col, qs) if col.numel() <= 16_000_000 else torch.quantile(col[:16_000_000], qs)
    allp = allgather_cat(pts.cpu()).permute(1, 0, 2).reshape(F, -1)  # [F, W * Q]
    cuts = []
    for f in range(F):
        v = allp[f]
        v = v[~torch.isnan(v)]
        if v.numel() == 0:
            cuts.append(torch.empty(0, device=X.device))
            continue
        u = torch.unique(v)
        if u.numel() > max_bin - 1:
            u = torch.unique(torch.quantile(v.double(), torch.linspace(0, 1, max_bin, dtype=torch.float64)[1:-1]).float())
            u = u[u > v.min()]
        else:
            u = u[1:]  # one bin per distinct value: cut at every value but the smallest
        cuts.append(u[: max_bin - 1].contiguous().to(X.device))
    return cuts


# ----------------------------------------------------------------------------- trees


class Tree:
    """Flat node arrays; node 0 is the root, ``left < 0`` marks a leaf. Split: go left iff
    ``x < thr`` (equivalently ``bin <= thr_bin``); missing values follow ``default_left``."""

    __slots__ = ("feature", "thr", "thr_bin", "default_left", "left", "right", "value", "gain", "cover", "depth",
                 "_cache")
    _FIELDS = ("feature", "thr", "thr_bin", "default_left", "left", "right", "value", "gain", "cover", "depth")

    def __init__(self):
        self.feature: List[int] = []
        self.thr: List[float] = []
        self.thr_bin: List[int] = []
        self.default_left: List[bool] = []
        self.left: List[int] = []
        self.right: List[int] = []
        self.value: List[float] = []
        self.gain: List[float] = []
        self.cover: List[float] = []
        self.depth = 0
        self._cache = None

    def add_node(self, value=0.0, cover=0.0) -> int:
        for a, v in ((self.feature, -1), (self.thr, 0.0), (self.thr_bin, 0), (self.default_left, True),
                     (self.left, -1), (self.right, -1), (self.value, value), (self.gain, 0.0), (self.cover, cover)):
            a.append(v)
        return len(self.feature) - 1

    @property
    def num_nodes(self) -> int:
        return len(self.feature)

    def to_dict(self) -> dict:
        return {k: getattr(self, k) for k in self._FIELDS}

    @classmethod
    def from_dict(cls, d: dict) -> "Tree":
        t = cls()
        for k in cls._FIELDS:
            setattr(t, k, d[k] if k == "depth" else list(d[k]))
        return t

    def tensors(self, device):
        key = (str(device), self.num_nodes)
        c = getattr(self, "_cache", None)
        if c is not None and c[0] == key:
            return c[1]
        i = torch.tensor([self.feature, self.thr_bin, self.default_left, self.left, self.right],
                         dtype=torch.long).to(device, non_blocking=True)
        fv = torch.tensor([self.thr, self.value], dtype=torch.float32).to(device, non_blocking=True)
        out = (i[0], fv[0], i[1], i[2].bool(), i[3], i[4], fv[1])
        self._cache = (key, out)
        return out

    def leaf_index_raw(self, X: torch.Tensor) -> torch.Tensor:
        feat, thr, _, dl, left, right, _ = self.tensors(X.device)
        node = torch.zeros(X.shape[0], dtype=torch.long, device=X.device)
        for _ in range(self.depth):
            lf = left[node]
            inner = lf >= 0
            x = X.gather(1, feat[node].clamp_min(0)[:, None])[:, 0]
            go_left = torch.where(torch.isnan(x), dl[node], x < thr[node])
            node = torch.where(inner, torch.where(go_left, lf, right[node]), node)
        return node

    def leaf_index_binned(self, bins: torch.Tensor, n: int) -> torch.Tensor:
        feat, _, tb, dl, left, right, _ = self.tensors(bins.device)
        node = torch.zeros(n, dtype=torch.long, device=bins.device)
        ar = torch.arange(n, device=bins.device)
        for _ in range(self.depth):
            lf = left[node]
            inner = lf >= 0
            b = bins[feat[node].clamp_min(0), ar].long()
            go_left = torch.where(b == MISSING_BIN, dl[node], b <= tb[node])
            node = torch.where(inner, torch.where(go_left, lf, right[node]), node)
        return node

    def predict_raw(self, X: torch.Tensor) -> torch.Tensor:
        return torch.tensor(self.value, dtype=torch.float32, device=X.device)[self.leaf_index_raw(X)]


# ----------------------------------------------------------------------------- objectives / metrics


def _grad_hess(obj: str, margin: torch.Tensor, y: torch.Tensor, w: Optional[torch.Tensor]):
    if obj == "squared":
        g, h = margin[:, 0] - y, torch.ones_like(y)
        g, h = g[:, None], h[:, None]
    elif obj in ("logistic", "logistic_raw"):
        p = torch.sigmoid(margin[:, 0])
        g, h = (p - y)[:, None], (p * (1 - p)).clamp_min(1e-16)[:, None]
    else:
        p = torch.softmax(margin, dim=1)
        oh = torch.nn.functional.one_hot(y.long(), margin.shape[1]).to(p.dtype)
        g, h = p - oh, (2.0 * p * (1 - p)).clamp_min(1e-16)
    if w is not None:
        g, h = g * w[:, None], h * w[:, None]
    return g, h


def transform(obj: str, margin: torch.Tensor) -> torch.Tensor:
    if obj == "squared" or obj == "logistic_raw":
        return margin[:, 0] if margin.shape[1] == 1 else margin
    if obj == "logistic":
        return torch.sigmoid(margin[:, 0])
    p = torch.softmax(margin, dim=1)
    return p.argmax(1).float() if obj == "softmax" else p


_EPS = 1e-15


_AUC_BINS = 1 << 16


def _auc(margin: torch.Tensor, y: torch.Tensor) -> float:
    """Distributed ROC AUC from score histograms: every worker bins its predicted probabilities
    (65536 bins) separately for positives and negatives, the histograms are all-reduced, and the
    AUC is the probability a random positive outscores a random negative (ties within a bin count
    1/2) -- exact up to the bin width, with no gather of the predictions."""
    p = torch.sigmoid(margin[:, 0]).clamp(0, 1)
    b = (p * (_AUC_BINS - 1)).round().long()
    pos = torch.bincount(b[y > 0.5], minlength=_AUC_BINS).double()
    neg = torch.bincount(b[y <= 0.5], minlength=_AUC_BINS).double()
    h = allreduce_sum(torch.stack([pos, neg]).cpu())
    pos, neg = h[0], h[1]
    P, N = float(pos.sum()), float(neg.sum())
    if P == 0 or N == 0:
        return float("nan")
    neg_below = torch.cumsum(neg, 0) - neg
    return float((pos * (neg_below + 0.5 * neg)).sum()) / (P * N)


def _metric_sums(name: str, obj: str, margin: torch.Tensor, y: torch.Tensor) -> Tuple[float, float]:
    """(sum of per-row loss, row count) for one metric; summed over workers by the caller."""
    n = float(y.numel())
    if name in ("rmse", "l2", "mse", "mae", "l1", "rmsle"):
        pred = transform(obj, margin) if obj != "softprob" else margin[:, 0]
        d = pred - y
        return (float((d * d).sum()) if name != "mae" and name != "l1" else float(d.abs().sum())), n
    if name in ("logloss", "binary_logloss"):
        p = torch.sigmoid(margin[:, 0]).clamp(_EPS, 1 - _EPS)
        return float(-(y * p.log() + (1 - y) * (1 - p).log()).sum()), n
    if name in ("error", "binary_error"):
        p = torch.sigmoid(margin[:, 0])
        return float(((p > 0.5).float() != y).float().sum()), n
    if name in ("mlogloss", "multi_logloss"):
        lp = torch.log_softmax(margin, dim=1).gather(1, y.long()[:, None])[:, 0]
        return float(-lp.clamp_min(math.log(_EPS)).sum()), n
    if name in ("merror", "multi_error"):
        return float((margin.argmax(1) != y.long()).float().sum()), n
    raise ValueError(f"unsupported eval metric {name!r}")


def _metric_finish(name: str, s: float, n: float) -> float:
    v = s / max(n, 1.0)
    return math.sqrt(v) if name == "rmse" else v


# ----------------------------------------------------------------------------- booster


class Booster:
    """Trained GBDT model: ``predict``, ``num_boosted_rounds``, ``save_model`` / ``load_model``
    (JSON), ``get_score`` feature importances, ``feature_names``."""

    def __init__(self, params: Optional[Dict[str, Any]] = None, flavor: str = "xgboost"):
        self.params = normalize_params(params, flavor) if params is None or "_obj" not in params else dict(params)
        self.trees: List[List[Tree]] = []  # [round][class]
        self.base_margin: List[float] = [0.0] * int(self.params["num_class"])
        self.cuts: Optional[List[List[float]]] = None
        self.feature_names: Optional[List[str]] = None
        self.best_iteration: Optional[int] = None
        self.best_score: Optional[float] = None

    # --- inference
    @property
    def num_class(self) -> int:
        return int(self.params["num_class"])

    def num_boosted_rounds(self) -> int:
        return len(self.trees)

    def num_features(self) -> int:
        return len(self.feature_names or [])

    def predict_margin(self, X: torch.Tensor, iteration_range: Optional[Tuple[int, int]] = None) -> torch.Tensor:
        K = self.num_class
        out = torch.tensor(self.base_margin, dtype=torch.float32, device=X.device).repeat(X.shape[0], 1)
        lo, hi = iteration_range or (0, len(self.trees))
        for rnd in self.trees[lo:hi]:
            for k in range(K):
                out[:, k] += rnd[k].predict_raw(X)
        return out

    def predict(self, data, output_margin: bool = False, iteration_range=None, device=None):
        """Predictions for ``data`` (DMatrix, numpy, pandas or torch). Returns numpy unless a torch
        tensor was passed."""
        is_t = isinstance(data, torch.Tensor)
        X = data.X if isinstance(data, DMatrix) else _to_tensor(data, device or (data.device if is_t else "cpu"))
        if X.dim() == 1:
            X = X[:, None]
        m = self.predict_margin(X, iteration_range)
        out = (m[:, 0] if m.shape[1] == 1 else m) if output_margin else transform(self.params["_obj"], m)
        return out if is_t else out.cpu().numpy()

    inplace_predict = predict

    def get_score(self, importance_type: str = "weight") -> Dict[str, float]:
        names = self.feature_names or []
        cnt: Dict[int, float] = {}
        gain: Dict[int, float] = {}
        cover: Dict[int, float] = {}
        for rnd in self.trees:
            for t in rnd:
                for i, f in enumerate(t.feature):
                    if t.left[i] >= 0:
                        cnt[f] = cnt.get(f, 0) + 1
                        gain[f] = gain.get(f, 0.0) + t.gain[i]
                        cover[f] = cover.get(f, 0.0) + t.cover[i]
        src = {"weight": cnt, "total_gain": gain, "total_cover": cover,
               "gain": {f: gain[f] / cnt[f] for f in cnt}, "cover": {f: cover[f] / cnt[f] for f in cnt}}
        if importance_type not in src:
            raise ValueError(f"importance_type {importance_type!r}")
        return {(names[f] if f < len(names) else f"f{f}"): float(v) for f, v in sorted(src[importance_type].items())}

    feature_importance = get_score

    # --- persistence
    def to_dict(self) -> dict:
        p = {k: v for k, v in self.params.items()}
        return {"format": "rca-gbdt-1", "params": p, "base_margin": self.base_margin, "cuts": self.cuts,
                "feature_names": self.feature_names, "best_iteration": self.best_iteration,
                "best_score": self.best_score, "trees": [[t.to_dict() for t in rnd] for rnd in self.trees]}

    @classmethod
    def from_dict(cls, d: dict) -> "Booster":
        if d.get("format") != "rca-gbdt-1":
            raise ValueError("not a GBDT model file written by this framework")
        b = cls(d["params"])
        b.base_margin = list(d["base_margin"])
        b.cuts = d.get("cuts")
        b.feature_names = d.get("feature_names")
        b.best_iteration = d.get("best_iteration")
        b.best_score = d.get("best_score")
        b.trees = [[Tree.from_dict(t) for t in rnd] for rnd in d["trees"]]
        return b

    def save_model(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.to_dict(), f)

    def load_model(self, path: str) -> "Booster":
        with open(path) as f:
            other = Booster.from_dict(json.load(f))
        self.__dict__.update(other.__dict__)
        return self

    def copy(self) -> "Booster":
        return Booster.from_dict(json.loads(json.dumps(self.to_dict())))

    def __getitem__(self, sl: slice) -> "Booster":
        b = self.copy()
        b.trees = b.trees[sl]
        return b


# ----------------------------------------------------------------------------- training


class TrainingCallback:
    """xgboost.callback.TrainingCallback protocol: return True from ``after_iteration`` to stop."""

    def before_training(self, model):
        return model

    def after_training(self, model):
        return model

    def before_iteration(self, model, epoch, evals_log) -> bool:
        return False

    def after_iteration(self, model, epoch, evals_log) -> bool:
        return False


class _Grower:
    def __init__(self, p: Dict[str, Any], bins: torch.Tensor, n: int, F: int, count_channel: bool):
        self.p = p
        self.bins, self.n, self.F = bins, n, F
        self.C = 3 if count_channel else 2
        self.lam = float(p["lambda"])
        self.alpha = float(p["alpha"])
        self.gamma = float(p["gamma"])
        self.mcw = float(p["min_child_weight"])
        self.mdl = int(p["min_data_in_leaf"])
        self.eta = float(p["eta"])
        self.max_depth = int(p["max_depth"])
        self.ld = bins.shape[1]
        self.dev = bins.device

    def _T(self, G):
        if self.alpha == 0.0:
            return G
        return torch.sign(G) * (G.abs() - self.alpha).clamp_min(0)

    def _score(self, G, H):
        t = self._T(G)
        return t * t / (H + self.lam)

    def leaf_value(self, G: float, H: float) -> float:
        t = math.copysign(max(abs(G) - self.alpha, 0.0), G) if self.alpha else G
        return -t / (H + self.lam) * self.eta

    def hist(self, pos: torch.Tensor, gh: torch.Tensor, slots: torch.Tensor, L: int) -> torch.Tensor:
        """Reduced histograms of L nodes: ``slots[node id] = slot`` (-1 = skip)."""
        from ...ops import gbdt_histogram

        node = torch.where(pos >= 0, slots[pos.clamp_min(0)], torch.full_like(pos, -1)).to(torch.int32)
        h = gbdt_histogram(self.bins, node.contiguous(), gh, L, precision=str(self.p.get("hist_precision", "auto")))
        return allreduce_sum(h)

    def best_splits(self, H: torch.Tensor, fmask: torch.Tensor):
        """Best split of each node from its reduced histogram [S, F, 256, C]. Returns per node
        (gain, feature, thr_bin, default_left, G, Hs, (GL, HL) of the left child)."""
        H64 = H.double()
        G_ = H64[..., 0]
        Hh = H64[..., 1]
        Gm, Hm = G_[..., MISSING_BIN], Hh[..., MISSING_BIN]
        GLc = torch.cumsum(G_[..., :MISSING_BIN], -1)
        HLc = torch.cumsum(Hh[..., :MISSING_BIN], -1)
        Gt = GLc[:, 0, -1] + Gm[:, 0]
        Ht = HLc[:, 0, -1] + Hm[:, 0]
        parent = self._score(Gt, Ht)[:, None, None]
        gains, valids = [], []
        extra = []
        if self.C == 3:
            Cn = H64[..., 2]
            CLc = torch.cumsum(Cn[..., :MISSING_BIN], -1)
            Cm = Cn[..., MISSING_BIN]
            Ct = CLc[:, 0, -1] + Cm[:, 0]
        for dleft in (True, False):
            GL = GLc + (Gm[..., None] if dleft else 0)
            HL = HLc + (Hm[..., None] if dleft else 0)
            GR, HR = Gt[:, None, None] - GL, Ht[:, None, None] - HL
            ok = (HL >= self.mcw) & (HR >= self.mcw) & (HL > 0) & (HR > 0)
            if self.C == 3:
                CL = CLc + (Cm[..., None] if dleft else 0)
                CR = Ct[:, None, None] - CL
                ok &= (CL >= max(self.mdl, 1)) & (CR >= max(self.mdl, 1))
            g = self._score(GL, HL) + self._score(GR, HR) - parent
            fm = fmask[None, :, None] if fmask.dim() == 1 else fmask[:, :, None]
            g = torch.where(ok & fm, g, torch.full_like(g, -math.inf))
            gains.append(g)
            extra.append((GL, HL))
        both = torch.stack(gains, -1)  # [S, F, 255, 2]
        S = both.shape[0]
        flat = both.reshape(S, -1)
        best, arg = flat.max(1)
        d = arg % 2
        tb = (arg // 2) % MISSING_BIN
        f = arg // (2 * MISSING_BIN)
        sidx = torch.arange(S, device=H.device)
        GLs = torch.where(d == 0, extra[0][0][sidx, f, tb], extra[1][0][sidx, f, tb])
        HLs = torch.where(d == 0, extra[0][1][sidx, f, tb], extra[1][1][sidx, f, tb])
        # one device->host copy for all of it (each .cpu() is a sync)
        packed = torch.stack([best, f.double(), tb.double(), (d == 0).double(), Gt, Ht, GLs, HLs]).cpu()
        b_, f_, tb_, dl_, Gt_, Ht_, GL_, HL_ = packed.unbind(0)
        return (b_, f_.long(), tb_.long(), dl_.bool(), Gt_, Ht_, GL_, HL_)

    def _node_masks(self, nodes: List[int], tree_mask: torch.Tensor) -> torch.Tensor:
        """xgboost's nested column sampling: ``colsample_bylevel`` draws from the tree's columns
        once per depth, ``colsample_bynode`` from the level's columns at every split."""
        byl = float(self.p.get("colsample_bylevel", 1.0) or 1.0)
        byn = float(self.p.get("colsample_bynode", 1.0) or 1.0)
        if byl >= 1.0 and byn >= 1.0:
            return tree_mask
        seed, F = int(self.p["seed"]), tree_mask.numel()
        out = []
        for i in nodes:
            d = self._depth_of[i]
            lvl = _feature_mask(F, byl, self._round * 4099 + 7 * d + 1, seed + 17, tree_mask.device, tree_mask)
            out.append(_feature_mask(F, byn, self._round * 4099 * 131 + 2 * i + 3, seed + 29, tree_mask.device, lvl))
        return torch.stack(out)

    def grow(self, g: torch.Tensor, h: torch.Tensor, row_mask: Optional[torch.Tensor], fmask: torch.Tensor,
             cuts: List[torch.Tensor]) -> Tree:
        n, ld, dev = self.n, self.ld, self.dev
        gh = torch.zeros(ld, self.C, dtype=torch.float32, device=dev)
        gh[:n, 0], gh[:n, 1] = g, h
        if self.C == 3:
            gh[:n, 2] = 1.0
        pos = torch.full((ld,), -1, dtype=torch.long, device=dev)
        pos[:n] = 0
        if row_mask is not None:
            pos[:n] = torch.where(row_mask, pos[:n], torch.full_like(pos[:n], -1))
        tree = Tree()
        tree.add_node()
        lossguide = self.p["grow_policy"] == "lossguide"
        max_leaves = int(self.p["max_leaves"]) if lossguide else 0
        max_depth = self.max_depth if self.max_depth > 0 else (10 ** 6)
        depth_of = {0: 0}
        self._depth_of = depth_of
        self._round = getattr(self, "_round_no", 0)
        slots = torch.full((1,), 0, dtype=torch.long, device=dev)
        root_h = self.hist(pos, gh, slots, 1)
        hists = {0: root_h[0]}
        cand: Dict[int, tuple] = {}

        def evaluate(nodes: List[int]):
            if not nodes:
                return
            Hs = torch.stack([hists[i] for i in nodes])
            res = self.best_splits(Hs, self._node_masks(nodes, fmask))
            for j, i in enumerate(nodes):
                gain, f, tb, dl, Gt, Ht, GL, HL = (r[j] for r in res)
                tree.cover[i] = float(Ht)
                tree.value[i] = self.leaf_value(float(Gt), float(Ht))
                if depth_of[i] < max_depth and math.isfinite(float(gain)) and float(gain) > max(self.gamma, 1e-12):
                    cand[i] = (float(gain), int(f), int(tb), bool(dl), float(GL), float(HL), float(Gt), float(Ht))

        evaluate([0])
        n_leaves = 1
        while cand:
            if lossguide:
                if n_leaves >= max_leaves:
                    break
                i = max(cand, key=lambda k: (cand[k][0], -k))
                batch = [i]
            else:
                dmin = min(depth_of[k] for k in cand)
                batch = sorted(k for k in cand if depth_of[k] == dmin)
            # apply the splits of this batch
            kids = []
            for i in batch:
                gain, f, tb, dl, GL, HL, Gt, Ht = cand.pop(i)
                l = tree.add_node(self.leaf_value(GL, HL), HL)
                r = tree.add_node(self.leaf_value(Gt - GL, Ht - HL), Ht - HL)
                tree.feature[i], tree.thr_bin[i], tree.default_left[i] = f, tb, dl
                c = cuts[f]
                tree.thr[i] = float(c[tb]) if tb < c.numel() else math.inf
                tree.left[i], tree.right[i], tree.gain[i] = l, r, gain
                depth_of[l] = depth_of[r] = depth_of[i] + 1
                tree.depth = max(tree.depth, depth_of[l])
                kids.append((i, l, r))
                n_leaves += 1
            # route the rows of the split nodes
            split_now = [False] * tree.num_nodes
            for k in kids:
                split_now[k[0]] = True
            tabs = torch.tensor([tree.feature, tree.thr_bin, tree.default_left, tree.left, tree.right, split_now],
                                dtype=torch.long).to(dev, non_blocking=True)  # one host->device copy
            feat_t, tb_t, dl_t, l_t, r_t, is_split = tabs[0], tabs[1], tabs[2].bool(), tabs[3], tabs[4], tabs[5].bool()
            pc = pos.clamp_min(0)
            act = (pos >= 0) & is_split[pc]
            b = self.bins[feat_t[pc].clamp_min(0), torch.arange(ld, device=dev)].long()
            go_left = torch.where(b == MISSING_BIN, dl_t[pc], b <= tb_t[pc])
            pos = torch.where(act, torch.where(go_left, l_t[pc], r_t[pc]), pos)
            kid_ids = [c for k in kids for c in (k[1], k[2])]
            for k in kids:
                if depth_of[k[1]] >= max_depth:
                    hists.pop(k[0], None)
            kids = [k for k in kids if depth_of[k[1]] < max_depth]
            if not kids:  # every child is at the depth limit: leaves, no histograms needed
                continue
            kid_ids = [c for k in kids for c in (k[1], k[2])]
            # histograms: build the smaller child of each pair (global row counts), subtract for the other
            # size proxy = the children's global hessian sums (known on the host from the split; the row
            # count itself for squared error), so choosing needs no device round trip
            small, big = [], []
            for j, (p_, l, r) in enumerate(kids):
                if tree.cover[l] <= tree.cover[r]:
                    small.append(l); big.append((r, p_, l))
                else:
                    small.append(r); big.append((l, p_, r))
            slots = torch.full((tree.num_nodes,), -1, dtype=torch.long, device=dev)
            slots[torch.tensor(small, dtype=torch.long, device=dev)] = torch.arange(len(small), device=dev)
            hs = self.hist(pos, gh, slots, len(small))
            for j, s in enumerate(small):
                hists[s] = hs[j]
            for (o, p_, s) in big:
                hists[o] = hists[p_] - hists[s]
            for k in kids:
                hists.pop(k[0], None)
            evaluate(kid_ids)
        return tree


def _feature_mask(F: int, frac: float, rnd: int, seed: int, device, parent: Optional[torch.Tensor] = None
                  ) -> torch.Tensor:
    """``frac`` of the features (of ``parent``'s when given), seeded identically on every worker."""
    base = torch.ones(F, dtype=torch.bool) if parent is None else parent.cpu()
    if frac >= 1.0:
        return base.to(device)
    g = torch.Generator(device="cpu").manual_seed(seed * 1000003 + rnd)  # same on every worker
    idx = base.nonzero().squeeze(1)
    k = max(1, int(round(frac * idx.numel())))
    m = torch.zeros(F, dtype=torch.bool)
    m[idx[torch.randperm(idx.numel(), generator=g)[:k]]] = True
    return m.to(device)


def train(params: Dict[str, Any], dtrain: DMatrix, num_boost_round: int = 10,
          evals: Sequence[Tuple[DMatrix, str]] = (), evals_result: Optional[Dict] = None,
          xgb_model: Optional[Booster] = None, callbacks: Sequence[TrainingCallback] = (),
          early_stopping_rounds: Optional[int] = None, flavor: str = "xgboost", init_model=None,
          verbose_eval: bool = False, **_ignored) -> Booster:
    """``xgboost.train``-shaped entry point. In a torch.distributed job every worker passes its own
    shard; histograms and metrics are summed over workers and all end with the same model."""
    p = normalize_params(params, flavor) if "_obj" not in params else dict(params)
    base = xgb_model if xgb_model is not None else init_model
    if dtrain.y is None:
        raise ValueError("dtrain needs a label")
    dev = dtrain.device
    N, F = dtrain.X.shape
    K = int(p["num_class"])
    obj = p["_obj"]
    if base is not None:
        bst = base.copy()
        bst.params.update({k: v for k, v in p.items() if k not in ("num_class", "_obj")})
        cuts = [torch.tensor(c, dtype=torch.float32, device=dev) for c in bst.cuts]
    else:
        bst = Booster(p)
        bst.feature_names = list(dtrain.feature_names)
        cuts = sketch_cuts(dtrain.X, int(p["max_bin"]), int(p["seed"]))
        bst.cuts = [c.cpu().tolist() for c in cuts]
        y = dtrain.y
        sums = allreduce_sum(torch.tensor([float(y.sum()), float(y.numel())], dtype=torch.float64))
        mean = float(sums[0] / max(float(sums[1]), 1.0))
        if p.get("base_score") is not None:
            bs = float(p["base_score"])
            base_m = bs if obj in ("squared", "logistic_raw") else math.log(max(bs, 1e-7) / max(1 - bs, 1e-7))
        elif obj == "squared":
            base_m = mean
        elif obj in ("logistic", "logistic_raw"):
            m = min(max(mean, 1e-6), 1 - 1e-6)
            base_m = math.log(m / (1 - m))
        else:
            base_m = 0.0
        bst.base_margin = [base_m] * K
    bins = dtrain.binned(cuts)
    grower = _Grower(p, bins, N, F, count_channel=int(p["min_data_in_leaf"]) > 0)
    margin = bst.predict_margin(dtrain.X)
    eval_sets = [(d, name, d.binned(cuts) if d is not dtrain else bins, bst.predict_margin(d.X) if d is not dtrain else None)
                 for d, name in evals]
    eval_margins = [m for *_, m in eval_sets]
    evals_log: Dict[str, Dict[str, List[float]]] = {}
    cbs = list(callbacks)
    for cb in cbs:
        bst = cb.before_training(bst) or bst
    gen = torch.Generator(device="cpu").manual_seed(int(p["seed"]) * 7 + 13 + 7919 * (dist.get_rank() if _world() > 1 else 0))
    start = bst.num_boosted_rounds()
    best = (math.inf, -1)
    row_mask_keep = None
    for it in range(start, start + num_boost_round):
        if any(cb.before_iteration(bst, it, evals_log) for cb in cbs):
            break
        g, h = _grad_hess(obj, margin, dtrain.y, dtrain.w)
        sub = float(p["subsample"])
        freq = int(p.get("bagging_freq", p.get("subsample_freq", 0)) or 0)
        if p["_flavor"] == "lightgbm":  # lightgbm bags only with bagging_freq > 0, re-drawn every freq rounds
            if sub < 1.0 and freq > 0 and (it % freq == 0 or row_mask_keep is None):
                row_mask_keep = (torch.rand(N, generator=gen) < sub).to(dev)
            row_mask = row_mask_keep if sub < 1.0 and freq > 0 else None
        else:
            row_mask = (torch.rand(N, generator=gen) < sub).to(dev) if sub < 1.0 else None
        fmask = _feature_mask(F, float(p["colsample_bytree"]), it, int(p["seed"]), dev)
        grower._round_no = it
        rnd = []
        for k in range(K):
            t = grower.grow(g[:, k].contiguous(), h[:, k].contiguous(), row_mask, fmask, cuts)
            rnd.append(t)
            vals = torch.tensor(t.value, dtype=torch.float32, device=dev)
            margin[:, k] += vals[t.leaf_index_binned(bins, N)]
            for j, (d, name, db, _) in enumerate(eval_sets):
                if d is dtrain:
                    continue
                eval_margins[j][:, k] += vals[t.leaf_index_binned(db, d.num_row())]
        bst.trees.append(rnd)
        # metrics, summed over workers
        for j, (d, name, _, _) in enumerate(eval_sets):
            m = margin if d is dtrain else eval_margins[j]
            for met in p["eval_metric"]:
                if met == "auc":
                    evals_log.setdefault(name, {}).setdefault(met, []).append(_auc(m, d.y))
                    continue
                s, n = _metric_sums(met, obj, m, d.y)
                tot = allreduce_sum(torch.tensor([s, n], dtype=torch.float64))
                evals_log.setdefault(name, {}).setdefault(met, []).append(_metric_finish(met, float(tot[0]), float(tot[1])))
        if evals_result is not None:
            evals_result.clear()
            evals_result.update({k: {m: list(v) for m, v in d.items()} for k, d in evals_log.items()})
        stop = False
        for cb in cbs:
            stop |= bool(cb.after_iteration(bst, it, evals_log))
        if early_stopping_rounds and eval_sets:
            last_name = eval_sets[-1][1]
            met = p["eval_metric"][-1]
            v = evals_log[last_name][met][-1]
            higher = met in ("auc", "map", "ndcg")
            score = -v if higher else v
            if score < best[0]:
                best = (score, it)
                bst.best_iteration, bst.best_score = it, v
            elif it - best[1] >= int(early_stopping_rounds):
                stop = True
        if stop:
            break
    for cb in cbs:
        bst = cb.after_training(bst) or bst
    return bst
