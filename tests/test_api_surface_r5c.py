"""Round-5 API surface, part 3 (reference: rllib/models, rllib/execution, old-stack policy names,
data/aggregate.py AggregateFn + Quantile, experimental/channel reader/writer interfaces,
util/annotations.RayDeprecationWarning, util/client, air/integrations, autoscaler/sdk,
tune.search.optuna / hyperopt, train.base_trainer)."""
import importlib
import queue
import warnings

import numpy as np
import pytest

import ray_community_amd as ray


def test_custom_aggregate_fn_and_quantile(ray_start_regular):
    from ray_community_amd.data.aggregate import AggregateFn, Quantile

    ds = ray.data.from_items([{"g": i % 3, "v": i} for i in range(30)])
    mean_fn = AggregateFn(init=lambda k: [0, 0], accumulate_row=lambda a, r: [a[0] + r["v"], a[1] + 1],
                          merge=lambda a, b: [a[0] + b[0], a[1] + b[1]], finalize=lambda a: a[0] / a[1],
                          name="avg")
    rows = ds.groupby("g").aggregate(mean_fn, Quantile("v", q=0.5)).take_all()
    assert [(r["g"], r["avg"], r["quantile(v)"]) for r in rows] == [(0, 13.5, 13.5), (1, 14.5, 14.5),
                                                                     (2, 15.5, 15.5)]
    total = AggregateFn(lambda k: 0, lambda a, b: a + b, "total",
                        accumulate_block=lambda a, df: a + int(df["v"].sum()))
    assert ds.aggregate(total) == {"total": 435}
    with pytest.raises(ValueError):
        AggregateFn(init=lambda k: 0, merge=lambda a, b: a, name="x")  # no accumulate_*


def test_rllib_models_catalog():
    import torch

    from ray_community_amd.rllib.models import MODEL_DEFAULTS, ModelCatalog, TorchModelV2
    from ray_community_amd.rllib.utils.spaces import Box, Dict, Discrete

    obs, act = Box(-1, 1, (4,), np.float32), Discrete(3)
    dist, n = ModelCatalog.get_action_dist(act, {})
    model = ModelCatalog.get_model_v2(obs, act, n, {"fcnet_hiddens": [16]})
    logits, _ = model({"obs": torch.zeros(5, 4)})
    assert logits.shape == (5, 3) and model.value_function().shape == (5,)
    d = dist(logits)
    ent = d.entropy()
    assert d.sample().shape == (5,) and bool(((ent > 0) & (ent <= np.log(3.0) + 1e-6)).all())

    class Tiny(TorchModelV2, torch.nn.Module):
        def __init__(self, obs_space, action_space, num_outputs, model_config, name, scale=1.0):
            torch.nn.Module.__init__(self)
            TorchModelV2.__init__(self, obs_space, action_space, num_outputs, model_config, name)
            self.lin = torch.nn.Linear(4, num_outputs)
            self.scale = scale

        def forward(self, input_dict, state, seq_lens):
            return self.scale * self.lin(input_dict["obs"]), state

        def value_function(self):
            return torch.zeros(1)

    ModelCatalog.register_custom_model("tiny", Tiny)
    m = ModelCatalog.get_model_v2(obs, act, 3, {"custom_model": "tiny", "custom_model_config": {"scale": 2.0}})
    assert isinstance(m, Tiny) and m.scale == 2.0 and len(m.trainable_variables()) == 2
    pre = ModelCatalog.get_preprocessor_for_space(Dict({"a": Discrete(2), "b": Box(-1, 1, (3,), np.float32)}))
    assert pre.shape == (5,) and pre.transform({"a": 1, "b": np.zeros(3)}).tolist() == [0, 1, 0, 0, 0]
    assert MODEL_DEFAULTS["fcnet_hiddens"] == [256, 256]


def test_execution_helpers_drive_a_ppo_step(ray_start_regular):
    from ray_community_amd.rllib.algorithms.ppo import PPOConfig
    from ray_community_amd.rllib.execution import (MinibatchBuffer, SimpleReplayBuffer, standardize_fields,
                                                   synchronous_parallel_sample, train_one_step)
    from ray_community_amd.rllib.policy.sample_batch import SampleBatch

    algo = (PPOConfig().environment("CartPole-v1").env_runners(num_env_runners=1, num_envs_per_env_runner=2)
            .training(train_batch_size=128, minibatch_size=64, num_epochs=1)).build()
    try:
        frags = synchronous_parallel_sample(worker_set=algo.env_runner_group, max_env_steps=128, concat=False)
        assert sum(len(f) for f in frags) >= 128
        res = train_one_step(algo, frags)
        assert "default_policy" in res and res["default_policy"]
    finally:
        algo.stop()
    b = standardize_fields(SampleBatch({"advantages": np.arange(10, dtype=np.float32)}), ["advantages"])
    assert abs(float(b["advantages"].mean())) < 1e-6 and abs(float(b["advantages"].std()) - 1) < 1e-5
    rb = SimpleReplayBuffer(2)
    for i in range(3):
        rb.add_batch(i)
    assert len(rb) == 2 and rb.replay() in (1, 2)
    q = queue.Queue()
    q.put("a")
    mb = MinibatchBuffer(q, size=1, timeout=1, num_passes=2, init_num_passes=2)
    assert mb.get() == ("a", False) and mb.get() == ("a", True)


def test_old_stack_policy_names():
    from ray_community_amd.rllib.algorithms import dqn, ppo, sac
    from ray_community_amd.rllib.policy import TorchPolicy

    assert issubclass(ppo.PPOTorchPolicy, TorchPolicy) and issubclass(dqn.DQNTorchPolicy, TorchPolicy)
    assert issubclass(sac.SACTorchPolicy, TorchPolicy)
    with pytest.raises(ImportError):
        ppo.PPOTF2Policy(None, None, {})
    with pytest.raises(ImportError):
        sac.RNNSAC()
    assert not hasattr(ppo, "NotAPolicyName")


def test_channel_reader_writer_interfaces():
    from ray_community_amd.experimental.channel import (AwaitableBackgroundReader, Channel, SynchronousReader,
                                                        SynchronousWriter)

    a, b = Channel(1 << 12), Channel(1 << 12)
    try:
        w = SynchronousWriter([a, b])
        r = SynchronousReader([a, b])
        w.write({"x": 1})
        assert r.read(timeout=5) == [{"x": 1}, {"x": 1}]
        bg = AwaitableBackgroundReader([a])
        bg.start()
        a.write(7, timeout=5)
        assert bg.read(timeout=5) == [7]
        bg.close()
    finally:
        a.destroy()
        b.destroy()


def test_misc_module_paths_and_stubs():
    from ray_community_amd.util.annotations import Deprecated, RayDeprecationWarning

    @Deprecated(message="use g")
    def f():
        return 1

    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        assert f() == 1
    assert any(issubclass(w.category, RayDeprecationWarning) for w in rec)
    from ray_community_amd.util.client import RayAPIStub, num_connected_contexts

    assert num_connected_contexts() == 0 and not RayAPIStub().is_connected()
    for mod, cls in (("wandb", "WandbLoggerCallback"), ("mlflow", "MLflowLoggerCallback"),
                     ("comet", "CometLoggerCallback")):
        m = importlib.import_module(f"ray_community_amd.air.integrations.{mod}")
        with pytest.raises(ImportError):
            getattr(m, cls)()
    from ray_community_amd.autoscaler import sdk

    cfg = sdk.fillout_defaults({"cluster_name": "c"})
    assert cfg["provider"] == {"type": "local"} and cfg["head_node_type"] == "head"
    with pytest.raises(NotImplementedError):
        sdk.create_or_update_cluster("cluster.yaml")
    assert importlib.import_module("ray_community_amd.tune.search.optuna").OptunaSearch
    assert importlib.import_module("ray_community_amd.tune.search.hyperopt").HyperOptSearch
    assert importlib.import_module("ray_community_amd.train.base_trainer").BaseTrainer
    from ray_community_amd.tune.search.bohb import BOHB, TuneBOHB

    assert BOHB is TuneBOHB


def test_trial_preprocessor_dag_and_misc_methods(ray_start_regular, tmp_path):
    from ray_community_amd import tune
    from ray_community_amd._private.worker import get_dashboard_url
    from ray_community_amd.data.preprocessors import Preprocessor, StandardScaler
    from ray_community_amd.tune.tuner import Trial
    from ray_community_amd.util.state import warnings_on_slow_request

    seen = {}

    class _CB(tune.Callback):
        def on_trial_result(self, iteration, trials, trial, result, **info):
            seen["tag"] = trial.experiment_tag
            seen["analysis"] = trial.metric_analysis
            seen["path"] = trial.path

    def f(config):
        for i in range(3):
            tune.report({"v": i * config["a"]})

    tune.Tuner(f, param_space={"a": 2}, run_config=ray.train.RunConfig(storage_path=str(tmp_path),
                                                                       callbacks=[_CB()])).fit()
    assert seen["tag"] == "a=2" and seen["analysis"]["v"]["max"] >= 2 and seen["path"].startswith(str(tmp_path))
    t = Trial("abc", {"x": 1}, str(tmp_path / "t"), {"CPU": 1})
    t2 = Trial.from_json_state(t.get_json_state())
    assert t2.trial_id == "abc" and t2.config == {"x": 1} and not t2.is_finished()

    ds = ray.data.from_items([{"x": float(i)} for i in range(10)])
    sc = StandardScaler(["x"])
    assert sc.fit_status() == Preprocessor.FitStatus.NOT_FITTED
    with pytest.raises(RuntimeError):
        sc.transform_batch({"x": np.zeros(2)})
    sc.fit(ds)
    back = Preprocessor.deserialize(sc.serialize())
    out = back.transform_batch({"x": np.array([4.5])})
    assert isinstance(out, dict) and abs(float(out["x"][0])) < 1e-9 and back.fit_status() == "FITTED"

    @ray.remote
    def inc(x):
        return x + 1

    from ray_community_amd.dag import InputNode

    with InputNode() as inp:
        dag = inc.bind(inc.bind(inp))
    assert ray.get(dag.execute(1, _ray_cache_refs=True)) == 3
    assert len(dag.get_object_refs_from_last_execute()) >= 2
    assert dag.apply_functional([1, (2, {"k": 3})], lambda x: x > 1, lambda x: x * 10) == [1, (20, {"k": 30})]
    with warnings_on_slow_request(address="http://x", endpoint="/api", timeout=0.01, explain=True):
        pass
    assert get_dashboard_url() is None or ":" in get_dashboard_url()


def test_util_module_paths():
    from ray_community_amd.util import iter_metrics, rpdb, serialization_addons
    from ray_community_amd.util.debugpy import set_trace  # noqa: F401

    sm = iter_metrics.SharedMetrics()
    sm.get().counters["n"] += 2
    child = iter_metrics.SharedMetrics(parents=[])
    iter_metrics.SharedMetrics(sm.get(), parents=[child])
    assert child.get().counters["n"] == 2
    serialization_addons.apply(None)
    assert callable(rpdb.set_trace)
    for mod in ("dask", "spark", "horovod"):
        with pytest.raises(ImportError):
            importlib.import_module(f"ray_community_amd.util.{mod}")


def test_train_module_paths_and_predictors():
    import pandas as pd
    import torch

    from ray_community_amd.train import constants, context, error, session  # noqa: F401
    from ray_community_amd.train.predictor import Predictor, PredictorNotSerializableException
    from ray_community_amd.train.torch.torch_detection_predictor import TorchDetectionPredictor

    p = Predictor.from_pandas_udf(lambda df: df.assign(y=df["x"] * 2))
    assert p.predict({"x": [1, 2]})["y"].tolist() == [2, 4]
    with pytest.raises(PredictorNotSerializableException):
        import pickle

        pickle.dumps(p)
    assert constants.TRAIN_DATASET_KEY == "train" and issubclass(error.SessionMisuseError, Exception)

    class Det(torch.nn.Module):
        def forward(self, ims):
            return [{"boxes": torch.zeros(1, 4), "labels": torch.ones(1), "scores": torch.ones(1)} for _ in ims]

    out = TorchDetectionPredictor(Det()).predict(np.zeros((2, 3, 4, 4), np.float32))
    assert out["pred_boxes"].shape == (2,) and out["pred_boxes"][1].shape == (1, 4)
    for mod in ("lightning", "tensorflow", "horovod", "mosaic"):
        with pytest.raises(ImportError):
            importlib.import_module(f"ray_community_amd.train.{mod}")
    assert isinstance(pd.DataFrame({"a": [1]}), pd.DataFrame)


def test_tune_serve_experimental_module_paths(ray_start_regular, tmp_path, capsys):
    for mod in ("tune.callback", "tune.progress_reporter", "tune.result_grid", "tune.tune_config", "tune.error",
                "tune.syncer", "tune.constants", "tune.result", "tune.trainable", "serve.deployment",
                "serve.context", "experimental.locations", "experimental.dynamic_resources"):
        importlib.import_module(f"ray_community_amd.{mod}")
    from ray_community_amd import serve
    from ray_community_amd.experimental.tqdm_ray import tqdm
    from ray_community_amd.serve.autoscaling_policy import calculate_desired_num_replicas
    from ray_community_amd.tune.syncer import Syncer

    assert calculate_desired_num_replicas({"target_ongoing_requests": 2, "min_replicas": 1, "max_replicas": 3},
                                          9, 1) == 3
    (tmp_path / "a").mkdir()
    (tmp_path / "a" / "f.txt").write_text("x")
    assert Syncer().sync_up(str(tmp_path / "a"), str(tmp_path / "b")) and (tmp_path / "b" / "f.txt").exists()
    assert list(tqdm(range(4), desc="bar", flush_interval_s=0)) == [0, 1, 2, 3]
    assert "bar: 4/4" in capsys.readouterr().out

    @serve.deployment
    class M:
        def __init__(self):
            from ray_community_amd.serve.metrics import Counter

            self.c = Counter("rca_test_requests_total", tag_keys=("route",))

        def __call__(self, x):
            self.c.inc(1, tags={"route": "/"})
            return dict(self.c._default_tags)

    try:
        tags = serve.run(M.bind(), name="m", route_prefix=None).remote(1).result()
        assert tags["deployment"] == "M" and tags["application"] == "m" and tags["replica"]
    finally:
        serve.shutdown()


def test_runtime_env_accessors():
    from ray_community_amd.runtime_env import RuntimeEnv

    r = RuntimeEnv(env_vars={"A": "1"}, working_dir="/tmp/wd", conda="myenv")
    assert r.has_working_dir() and r.working_dir_uri() == "/tmp/wd" and r.has_conda()
    assert r.conda_env_name() == "myenv" and not r.has_pip() and r.plugin_uris() == []
    r.set("env_vars", {"B": "2"})
    assert r.env_vars() == {"B": "2"}
    with pytest.raises(ValueError):
        r.set("not_a_field", 1)
