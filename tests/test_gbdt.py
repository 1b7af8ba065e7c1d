"""Native data-parallel GBDT behind train.xgboost / train.lightgbm, and train.sklearn.

Reference test models: python/ray/train/tests/test_xgboost_trainer.py (fit with train + valid
datasets, metrics reported as ``{name}-{metric}``, resume trains the remaining rounds, checkpoint
frequency / at end, predictor on the checkpoint), test_lightgbm_trainer.py, test_sklearn_predictor.py.
xgboost / lightgbm are not installed: model quality is pinned against sklearn's
HistGradientBoosting on the same data instead ("parity unpinned" against the libraries themselves).
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

from ray_community_amd import ops
from ray_community_amd.train.gbdt import Booster, DMatrix, TrainingCallback, train
from ray_community_amd.train.gbdt.core import MISSING_BIN


def _reg(n=3000, f=6, seed=0, nan=0.0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, f)).astype(np.float32)
    y = (2 * X[:, 0] + np.sin(2 * X[:, 1]) + 0.5 * X[:, 2] * X[:, 3] + rng.normal(scale=0.1, size=n)).astype(np.float32)
    if nan:
        X[rng.random(X.shape) < nan] = np.nan
    return X, y


def test_histogram_cpu_matches_dense_reference():
    rng = np.random.default_rng(1)
    F, n, L = 3, 103, 4
    ld = (n + 3) // 4 * 4
    bins = torch.full((F, ld), MISSING_BIN, dtype=torch.uint8)
    bins[:, :n] = torch.as_tensor(rng.integers(0, 256, size=(F, n)), dtype=torch.uint8)
    node = torch.full((ld,), -1, dtype=torch.int32)
    node[:n] = torch.as_tensor(rng.integers(-1, L, size=n), dtype=torch.int32)
    gh = torch.zeros(ld, 3)
    gh[:n] = torch.as_tensor(rng.normal(size=(n, 3)), dtype=torch.float32)
    h = ops.gbdt_histogram(bins, node, gh, L)
    ref = torch.zeros(L, F, 256, 3, dtype=torch.float64)
    for r in range(n):
        if node[r] >= 0:
            for f in range(F):
                ref[int(node[r]), f, int(bins[f, r])] += gh[r].double()
    torch.testing.assert_close(h.double(), ref, rtol=1e-5, atol=1e-5)


def test_regression_quality_close_to_sklearn_hist_gbdt():
    from sklearn.ensemble import HistGradientBoostingRegressor

    X, y = _reg(4000)
    res = {}
    b = train({"objective": "reg:squarederror", "max_depth": 5, "eta": 0.3, "lambda": 0.0},
              DMatrix(X[:3000], y[:3000]), 40, evals=[(DMatrix(X[3000:], y[3000:]), "valid")], evals_result=res)
    ours = float(np.sqrt(np.mean((b.predict(X[3000:]) - y[3000:]) ** 2)))
    assert abs(ours - res["valid"]["rmse"][-1]) < 1e-4  # raw-feature predict == binned training traversal
    sk = HistGradientBoostingRegressor(max_iter=40, learning_rate=0.3, max_depth=5, early_stopping=False)
    sk = float(np.sqrt(np.mean((sk.fit(X[:3000], y[:3000]).predict(X[3000:]) - y[3000:]) ** 2)))
    assert ours < 1.15 * sk, (ours, sk)
    assert res["valid"]["rmse"][-1] < res["valid"]["rmse"][0]


def test_missing_values_learn_default_direction():
    rng = np.random.default_rng(2)
    x = rng.normal(size=2000).astype(np.float32)
    y = (x > 0).astype(np.float32) * 3.0
    miss = rng.random(2000) < 0.3
    y[miss] = 5.0  # missing rows have their own target: a default direction must route them
    x[miss] = np.nan
    b = train({"objective": "reg:squarederror", "max_depth": 3, "eta": 1.0, "lambda": 0.0}, DMatrix(x[:, None], y), 3)
    p = b.predict(np.array([[np.nan], [-1.0], [1.0]], dtype=np.float32))
    np.testing.assert_allclose(p, [5.0, 0.0, 3.0], atol=0.05)


def test_binary_and_multiclass_objectives():
    rng = np.random.default_rng(3)
    X = rng.normal(size=(3000, 4)).astype(np.float32)
    yb = (X[:, 0] + X[:, 1] > 0).astype(np.float32)
    res = {}
    b = train({"objective": "binary:logistic", "eval_metric": ["logloss", "error"]}, DMatrix(X, yb), 20,
              evals=[(DMatrix(X, yb), "train")], evals_result=res)
    p = b.predict(X)
    assert ((p > 0.5) == (yb > 0.5)).mean() > 0.95 and res["train"]["error"][-1] < 0.05
    assert 0 <= p.min() and p.max() <= 1
    yc = np.digitize(X[:, 0], [-0.5, 0.5]).astype(np.float32)
    bc = train({"objective": "multi:softprob", "num_class": 3}, DMatrix(X, yc), 15)
    pc = bc.predict(X)
    assert pc.shape == (3000, 3) and np.allclose(pc.sum(1), 1, atol=1e-5)
    assert (pc.argmax(1) == yc).mean() > 0.95
    bs = train({"objective": "multi:softmax", "num_class": 3}, DMatrix(X, yc), 15)
    assert set(np.unique(bs.predict(X))) <= {0.0, 1.0, 2.0}


def test_lossguide_respects_num_leaves_and_lightgbm_defaults():
    X, y = _reg(2000)
    b = train({"objective": "regression", "num_leaves": 7}, DMatrix(X, y), 5, flavor="lightgbm")
    assert b.params["eta"] == 0.1 and b.params["grow_policy"] == "lossguide"
    for rnd in b.trees:
        leaves = sum(1 for l in rnd[0].left if l < 0)
        assert 2 <= leaves <= 7
    # min_data_in_leaf (lightgbm default 20): every leaf covers >= 20 rows
    leaf = rnd[0].leaf_index_raw(torch.as_tensor(X))
    assert torch.bincount(leaf)[torch.bincount(leaf) > 0].min() >= 20


def test_save_load_roundtrip_importance_and_continue(tmp_path):
    X, y = _reg(1500, nan=0.05)
    d = DMatrix(pd.DataFrame(X, columns=[f"c{i}" for i in range(X.shape[1])]), y)
    b = train({"max_depth": 4}, d, 6)
    path = os.path.join(tmp_path, "m.json")
    b.save_model(path)
    b2 = Booster().load_model(path)
    np.testing.assert_array_equal(b.predict(X), b2.predict(X))
    imp = b2.get_score(importance_type="gain")
    assert max(imp, key=imp.get) == "c0" and b2.feature_names[0] == "c0"
    b3 = train({"max_depth": 4}, d, 4, xgb_model=b2)
    assert b3.num_boosted_rounds() == 10
    np.testing.assert_array_equal(b3[:6].predict(X), b.predict(X))


def test_early_stopping_and_callbacks():
    X, y = _reg(1200)
    rng = np.random.default_rng(9)
    yn = rng.normal(size=y.shape).astype(np.float32)  # pure noise validation target: stops early

    class Count(TrainingCallback):
        def __init__(self):
            self.n = 0

        def after_iteration(self, model, epoch, evals_log):
            self.n += 1
            return False

    cb = Count()
    b = train({"max_depth": 6, "eta": 0.5}, DMatrix(X[:800], y[:800]), 200,
              evals=[(DMatrix(X[800:], yn[800:]), "valid")], early_stopping_rounds=3, callbacks=[cb])
    assert b.num_boosted_rounds() < 50 and cb.n == b.num_boosted_rounds()
    assert b.best_iteration is not None and b.best_iteration <= b.num_boosted_rounds() - 1


def _dist_worker(rank, world, port, X, y, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sl = slice(rank * len(X) // world, (rank + 1) * len(X) // world)
    res = {}
    b = train({"max_depth": 4, "subsample": 0.8, "colsample_bytree": 0.8}, DMatrix(X[sl], y[sl]), 8,
              evals=[(DMatrix(X[sl], y[sl]), "train")], evals_result=res)
    q.put((rank, b.to_dict(), res["train"]["rmse"][-1]))
    dist.destroy_process_group()


def test_data_parallel_workers_build_identical_models():
    import socket

    import torch.multiprocessing as mp

    X, y = _reg(2000)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, X, y, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    (_, m0, r0), (_, m1, r1) = out
    assert m0["trees"] == m1["trees"] and m0["cuts"] == m1["cuts"] and r0 == r1
    b = Booster.from_dict(m0)
    assert np.sqrt(np.mean((b.predict(X) - y) ** 2)) < 0.6 * np.std(y)


@pytest.fixture
def ray4():
    import ray_community_amd as ray

    ray.init(num_cpus=4, log_to_driver=False)
    yield
    ray.shutdown()


def test_xgboost_trainer_fit_resume_predict(ray4, tmp_path):
    from ray_community_amd import data
    from ray_community_amd.train import CheckpointConfig, RunConfig, ScalingConfig
    from ray_community_amd.train.xgboost import XGBoostPredictor, XGBoostTrainer

    X, y = _reg(2400, f=4)
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    df["y"] = y
    tr, va = data.from_pandas(df.iloc[:2000]), data.from_pandas(df.iloc[2000:])
    with pytest.raises(KeyError):
        XGBoostTrainer(label_column="y", params={}, datasets={"valid": va})
    res = XGBoostTrainer(label_column="y", params={"objective": "reg:squarederror", "max_depth": 4},
                         num_boost_round=8, scaling_config=ScalingConfig(num_workers=2),
                         datasets={"train": tr, "valid": va},
                         run_config=RunConfig(name="xgb", storage_path=str(tmp_path),
                                              checkpoint_config=CheckpointConfig(checkpoint_frequency=4))).fit()
    assert {"train-rmse", "valid-rmse"} <= set(res.metrics)
    model = XGBoostTrainer.get_model(res.checkpoint)
    assert model.num_boosted_rounds() == 8
    pred = XGBoostPredictor.from_checkpoint(res.checkpoint).predict(df.iloc[2000:].drop(columns=["y"]))
    rmse = float(np.sqrt(np.mean((pred["predictions"].to_numpy() - y[2000:]) ** 2)))
    assert abs(rmse - res.metrics["valid-rmse"]) < 1e-3
    hist = res.metrics_dataframe
    assert list(hist["valid-rmse"])[0] > list(hist["valid-rmse"])[-1]
    # num_boost_round is the TARGET: resuming from an 8-round model trains 4 more
    res2 = XGBoostTrainer(label_column="y", params={"objective": "reg:squarederror", "max_depth": 4},
                          num_boost_round=12, scaling_config=ScalingConfig(num_workers=2),
                          datasets={"train": tr, "valid": va}, resume_from_checkpoint=res.checkpoint,
                          run_config=RunConfig(name="xgb2", storage_path=str(tmp_path))).fit()
    assert XGBoostTrainer.get_model(res2.checkpoint).num_boosted_rounds() == 12
    assert res2.metrics["valid-rmse"] <= res.metrics["valid-rmse"] + 1e-6


def test_lightgbm_trainer_binary(ray4, tmp_path):
    from ray_community_amd import data
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.lightgbm import LightGBMPredictor, LightGBMTrainer

    rng = np.random.default_rng(4)
    X = rng.normal(size=(2000, 3))
    df = pd.DataFrame(X, columns=["u", "v", "w"])
    df["label"] = (X[:, 0] - X[:, 2] > 0).astype(int)
    res = LightGBMTrainer(label_column="label", params={"objective": "binary", "metric": ["binary_logloss",
                                                                                          "binary_error"]},
                          num_boost_round=15, scaling_config=ScalingConfig(num_workers=2),
                          datasets={"train": data.from_pandas(df)},
                          run_config=RunConfig(name="lgb", storage_path=str(tmp_path))).fit()
    assert res.metrics["train-binary_error"] < 0.08
    p = LightGBMPredictor.from_checkpoint(res.checkpoint).predict(df.drop(columns=["label"]))
    assert ((p["predictions"].to_numpy() > 0.5) == df["label"].to_numpy()).mean() > 0.92


def test_sklearn_checkpoint_predictor_and_deprecated_trainer(tmp_path):
    from sklearn.linear_model import LinearRegression

    from ray_community_amd.data.preprocessors import StandardScaler
    from ray_community_amd.train.sklearn import SklearnCheckpoint, SklearnPredictor, SklearnTrainer

    with pytest.raises(DeprecationWarning):
        SklearnTrainer(estimator=None)
    X = np.arange(20, dtype=float).reshape(10, 2)
    y = X @ np.array([1.0, 2.0]) + 3
    est = LinearRegression().fit(X, y)
    ck = SklearnCheckpoint.from_estimator(est, path=str(tmp_path / "ck"))
    pr = SklearnPredictor.from_checkpoint(ck)
    np.testing.assert_allclose(pr.predict(X)["predictions"], y)
    df = pd.DataFrame(X, columns=["a", "b"])
    out = pr.predict(df)
    assert list(out.columns) == ["predictions"]
    np.testing.assert_allclose(out["predictions"], y)
    assert isinstance(ck.get_estimator(), LinearRegression) and ck.get_preprocessor() is None


# ----------------------------------------------------------------------------- GPU


@pytest.mark.gpu
def test_gbdt_hist_kernel_matches_cpu_reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(5)
    for F, n, L, C in ((7, 100_003, 3, 2), (2, 50_001, 40, 3), (33, 20_000, 1, 2)):
        ld = (n + 3) // 4 * 4
        bins = torch.full((F, ld), MISSING_BIN, dtype=torch.uint8)
        bins[:, :n] = torch.as_tensor(rng.integers(0, 256, size=(F, n)), dtype=torch.uint8)
        node = torch.full((ld,), -1, dtype=torch.int32)
        node[:n] = torch.as_tensor(rng.integers(-1, L, size=n), dtype=torch.int32)
        gh = torch.zeros(ld, C)
        gh[:n, 0] = torch.as_tensor(rng.normal(size=n), dtype=torch.float32)
        gh[:n, 1] = torch.as_tensor(rng.random(size=n), dtype=torch.float32)  # hessians are >= 0
        if C == 3:
            gh[:n, 2] = 1.0  # row count channel
        ref = ops.gbdt_histogram(bins, node, gh, L)  # CPU index_add reference
        got = ops.gbdt_histogram(bins.cuda(), node.cuda(), gh.cuda(), L)
        torch.cuda.synchronize()
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=2e-3)  # fixed-point (grad, hess) on the GPU


@pytest.mark.gpu
def test_gbdt_training_on_gpu_matches_cpu_quality():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    X, y = _reg(20_000, f=8, nan=0.02)
    res_c, res_g = {}, {}
    bc = train({"max_depth": 6}, DMatrix(X, y), 10, evals=[(DMatrix(X, y), "train")], evals_result=res_c)
    dg = DMatrix(X, y, device="cuda")
    bg = train({"max_depth": 6}, dg, 10, evals=[(dg, "train")], evals_result=res_g)
    # float atomics reorder sums: splits may differ on near-ties, the fit may not
    assert abs(res_c["train"]["rmse"][-1] - res_g["train"]["rmse"][-1]) < 0.02 * res_c["train"]["rmse"][-1]
    assert bg.trees[0][0].feature[0] == bc.trees[0][0].feature[0]
    p = bg.predict(torch.as_tensor(X, device="cuda"))
    assert p.is_cuda and abs(float(torch.sqrt(torch.mean((p.cpu() - torch.as_tensor(y)) ** 2)))
                             - res_g["train"]["rmse"][-1]) < 1e-3


def test_tuner_searches_xgboost_params(ray4, tmp_path):
    """``Tuner(XGBoostTrainer(...), param_space={"params": {...}})`` as in the reference's GBDT
    tuning examples: each trial trains with its own booster parameters."""
    from ray_community_amd import data, tune
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.xgboost import XGBoostTrainer

    X, y = _reg(1500, f=4)
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    df["y"] = y
    trainer = XGBoostTrainer(label_column="y", params={"objective": "reg:squarederror"}, num_boost_round=6,
                             scaling_config=ScalingConfig(num_workers=1),
                             datasets={"train": data.from_pandas(df.iloc[:1200]),
                                       "valid": data.from_pandas(df.iloc[1200:])})
    grid = tune.Tuner(trainer, param_space={"params": {"max_depth": tune.grid_search([1, 5])}},
                      tune_config=tune.TuneConfig(metric="valid-rmse", mode="min"),
                      run_config=RunConfig(name="tune_xgb", storage_path=str(tmp_path))).fit()
    assert len(grid) == 2 and not grid.errors
    best = grid.get_best_result()
    assert best.config["params"]["max_depth"] == 5
    scores = sorted(r.metrics["valid-rmse"] for r in grid)
    assert scores[0] < scores[1]
    assert XGBoostTrainer.get_model(best.checkpoint).trees[0][0].depth == 5


def test_auc_metric_matches_sklearn_and_drives_early_stopping():
    from sklearn.metrics import roc_auc_score

    rng = np.random.default_rng(3)
    X = rng.normal(size=(4000, 4)).astype(np.float32)
    y = ((X[:, 0] + rng.normal(size=4000)) > 0).astype(np.float32)
    res = {}
    dv = DMatrix(X[3000:], y[3000:])
    b = train({"objective": "binary:logistic", "eval_metric": ["logloss", "auc"]}, DMatrix(X[:3000], y[:3000]), 60,
              evals=[(dv, "valid")], evals_result=res, early_stopping_rounds=5)
    assert abs(res["valid"]["auc"][-1] - roc_auc_score(y[3000:], b.predict(X[3000:]))) < 1e-4
    # auc is the last metric -> early stopping maximises it
    assert b.best_score == max(res["valid"]["auc"]) and b.num_boosted_rounds() < 60


@pytest.mark.gpu
def test_xgboost_trainer_on_gpu_worker(tmp_path):
    """The trainer path end to end on a GPU worker: shard -> HBM DMatrix -> HIP histograms."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ray_community_amd as ray
    from ray_community_amd import data
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.xgboost import XGBoostTrainer

    ray.init(num_cpus=4, num_gpus=1, log_to_driver=False)
    try:
        rng = np.random.default_rng(6)
        X = rng.normal(size=(20_000, 6))
        df = pd.DataFrame(X, columns=[f"f{i}" for i in range(6)])
        df["label"] = ((X[:, 0] + 0.5 * X[:, 1] ** 2) > 0.5).astype(float)

        def dev_probe(batch):
            return batch

        res = XGBoostTrainer(label_column="label",
                             params={"objective": "binary:logistic", "eval_metric": ["error", "auc"]},
                             num_boost_round=10, scaling_config=ScalingConfig(num_workers=1, use_gpu=True),
                             datasets={"train": data.from_pandas(df.iloc[:16000]).map_batches(dev_probe),
                                       "valid": data.from_pandas(df.iloc[16000:])},
                             run_config=RunConfig(name="xgb_gpu", storage_path=str(tmp_path))).fit()
        assert res.metrics["valid-error"] < 0.1 and res.metrics["valid-auc"] > 0.95
        assert XGBoostTrainer.get_model(res.checkpoint).num_boosted_rounds() == 10
    finally:
        ray.shutdown()


def test_xgboost_trainer_v2_form_with_user_loop(ray4, tmp_path):
    """Reference v2 form: ``XGBoostTrainer(train_loop_per_worker, xgboost_config=...)``, the loop
    trains on its shard with ``train(...)`` and ``RayTrainReportCallback``."""
    from ray_community_amd import data, train as rtrain
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.xgboost import RayTrainReportCallback, XGBoostConfig, XGBoostTrainer
    from ray_community_amd.train.xgboost import train as xtrain

    X, y = _reg(1600, f=4)
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    df["y"] = y

    def loop(config):
        shard = rtrain.get_dataset_shard("train").materialize().to_pandas()
        d = DMatrix(shard.drop(columns=["y"]), label=shard["y"])
        xtrain(config, d, num_boost_round=config["rounds"], evals=[(d, "train")],
               callbacks=[RayTrainReportCallback(metrics={"loss": "train-rmse"}, frequency=2)])

    res = XGBoostTrainer(loop, train_loop_config={"max_depth": 3, "rounds": 4},
                         xgboost_config=XGBoostConfig(), scaling_config=ScalingConfig(num_workers=2),
                         datasets={"train": data.from_pandas(df)},
                         run_config=RunConfig(name="v2", storage_path=str(tmp_path))).fit()
    assert set(res.metrics) >= {"loss"} and res.metrics["loss"] < np.std(y)
    assert RayTrainReportCallback.get_model(res.checkpoint).num_boosted_rounds() == 4


def test_column_sampling_levels_and_lightgbm_bagging_freq():
    X, y = _reg(1500, f=6)
    # colsample_bynode: every split draws its own columns -> the strong feature 0 cannot win every split
    b = train({"max_depth": 3, "colsample_bynode": 0.34, "seed": 3}, DMatrix(X, y), 6)
    full = train({"max_depth": 3}, DMatrix(X, y), 6)
    roots_full = {r[0].feature[0] for r in full.trees}
    roots = {r[0].feature[0] for r in b.trees}
    assert roots_full == {0} and len(roots) > 1
    again = train({"max_depth": 3, "colsample_bynode": 0.34, "seed": 3}, DMatrix(X, y), 6)
    assert again.to_dict()["trees"] == b.to_dict()["trees"]  # seeded, reproducible
    lv = train({"max_depth": 3, "colsample_bylevel": 0.5, "seed": 1}, DMatrix(X, y), 4)
    assert lv.num_boosted_rounds() == 4
    # lightgbm: bagging_fraction alone does nothing (bagging_freq defaults to 0)
    a = train({"objective": "regression", "bagging_fraction": 0.5}, DMatrix(X, y), 3, flavor="lightgbm")
    c = train({"objective": "regression"}, DMatrix(X, y), 3, flavor="lightgbm")
    assert a.to_dict()["trees"] == c.to_dict()["trees"]
    d = train({"objective": "regression", "bagging_fraction": 0.5, "bagging_freq": 1}, DMatrix(X, y), 3,
              flavor="lightgbm")
    assert d.to_dict()["trees"] != c.to_dict()["trees"]


def test_histogram_exact_precision_cpu():
    """precision="exact" on the CPU: fp64 accumulation rounded once (the GPU exact kernel's
    numbers); "auto" on the CPU keeps the plain fp32 path."""
    rng = np.random.default_rng(2)
    F, n, L = 4, 4001, 3
    ld = (n + 3) // 4 * 4
    bins = torch.as_tensor(rng.integers(0, 256, size=(F, ld)), dtype=torch.uint8)
    node = torch.as_tensor(rng.integers(-1, L, size=ld), dtype=torch.int32)
    gh = torch.as_tensor(rng.normal(size=(ld, 2)) * 10.0 ** rng.integers(-6, 3, size=(ld, 2)), dtype=torch.float32)
    ex = ops.gbdt_histogram(bins, node, gh, L, precision="exact")
    ref = torch.zeros(L * F * 256, 2, dtype=torch.float64)
    keep = node >= 0
    idx = ((node[keep].long()[None] * F + torch.arange(F)[:, None]) * 256 + bins[:, keep].long()).reshape(-1)
    ref.index_add_(0, idx, gh[keep].double().unsqueeze(0).expand(F, -1, -1).reshape(-1, 2))
    assert torch.equal(ex.view(-1, 2), ref.float())
    with pytest.raises(ValueError):
        ops.gbdt_histogram(bins, node, gh, L, precision="bf16")


def _heavy_tailed_logistic(n, F, L, seed=7):
    """Logistic-loss statistics with confident rows: hessians p(1-p) spanning ~6 binades."""
    rng = np.random.default_rng(seed)
    ld = (n + 3) // 4 * 4
    bins = torch.full((F, ld), MISSING_BIN, dtype=torch.uint8)
    bins[:, :n] = torch.as_tensor(rng.integers(0, 64, size=(F, n)), dtype=torch.uint8)
    node = torch.full((ld,), -1, dtype=torch.int32)
    node[:n] = torch.as_tensor(rng.integers(0, L, size=n), dtype=torch.int32)
    margin = rng.normal(scale=6.0, size=n)
    p = 1.0 / (1.0 + np.exp(-margin))
    y = rng.random(n) < p
    gh = torch.zeros(ld, 2)
    gh[:n, 0] = torch.as_tensor(p - y, dtype=torch.float32)
    gh[:n, 1] = torch.as_tensor(p * (1 - p), dtype=torch.float32)
    return bins, node, gh


@pytest.mark.gpu
def test_gbdt_exact_histograms_gpu_match_cpu_on_heavy_tailed_hessians():
    """Exact mode: GPU histograms equal the CPU fp64 ones (to the last fp32 ulp). With hessians
    spanning ~1e-6..0.25 "auto" switches to the exact kernel, which is closer to the reference
    than the fixed-point one."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    bins, node, gh = _heavy_tailed_logistic(200_003, 5, 6)
    ref = ops.gbdt_histogram(bins, node, gh, 6, precision="exact")
    got = ops.gbdt_histogram(bins.cuda(), node.cuda(), gh.cuda(), 6, precision="exact").cpu()
    torch.testing.assert_close(got, ref, rtol=2e-7, atol=1e-12)
    fixed = ops.gbdt_histogram(bins.cuda(), node.cuda(), gh.cuda(), 6, precision="fixed").cpu()
    small = ref[..., 1] > 0
    rel = lambda h: ((h[..., 1] - ref[..., 1]).abs() / ref[..., 1].clamp_min(1e-30))[small].max().item()
    # the fixed-point kernel quantises each hessian (its bin sums are off by ~1e-6 relative here,
    # measured); the exact kernel is closer to the fp64 reference
    assert rel(got) < rel(fixed)
    assert ops._gbdt_needs_exact(gh.cuda())
    auto = ops.gbdt_histogram(bins.cuda(), node.cuda(), gh.cuda(), 6).cpu()
    torch.testing.assert_close(auto, ref, rtol=2e-7, atol=1e-12)


@pytest.mark.gpu
def test_gbdt_exact_mode_grows_the_same_trees_on_gpu_and_cpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    X, y = _reg(20_000, f=8, nan=0.02)
    params = {"max_depth": 5, "hist_precision": "exact"}
    bc = train(params, DMatrix(X, y), 8)
    bg = train(params, DMatrix(X, y, device="cuda"), 8)
    for tc, tg in zip(bc.trees, bg.trees):
        assert list(tc[0].feature) == list(tg[0].feature)
    pc = bc.predict(torch.as_tensor(X))
    pg = bg.predict(torch.as_tensor(X, device="cuda")).cpu()
    torch.testing.assert_close(pg, pc, rtol=1e-5, atol=1e-5)
