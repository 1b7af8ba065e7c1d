"""Reference API surface added in round 5 (class-level methods user code calls or overrides):
SampleBatch (rllib/policy/sample_batch.py), Algorithm (rllib/algorithms/algorithm.py), Tune's
Trainable / Searcher / TrialScheduler, MultiAgentEnv helpers + BaseEnv conversion, Serve
Deployment properties."""
import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd.rllib.policy.sample_batch import SampleBatch


def test_sample_batch_reference_methods():
    b = SampleBatch({"a": np.array([1, 2, 3]), "seq_lens": np.array([1, 2])})
    assert b.right_zero_pad(max_seq_len=4)["a"].tolist() == [1, 0, 0, 0, 2, 3, 0, 0]
    assert b.zero_padded and b.max_seq_len == 4
    e = SampleBatch({"obs": np.arange(6).reshape(6, 1), "new_obs": np.arange(1, 7).reshape(6, 1),
                     "eps_id": np.array([1, 1, 2, 2, 2, 3]), "terminateds": np.array([0, 1, 0, 0, 1, 0], bool)})
    assert [x.count for x in e.split_by_episode()] == [2, 3, 1]
    assert not e.is_single_trajectory() and e.split_by_episode()[0].is_single_trajectory()
    assert e.split_by_episode()[1].is_terminated_or_truncated()
    rows = list(e.rows())
    assert len(rows) == 6 and rows[2]["eps_id"] == 2
    assert e.size_bytes() == sum(v.nbytes for v in e.values())
    c = e.copy().compress()
    assert isinstance(c["obs"][0], bytes)
    assert np.array_equal(c.decompress_if_needed()["obs"], e["obs"])
    assert e.concat(e).count == 12 and SampleBatch.concat_samples([e, e, e]).count == 18
    step = e.get_single_step_input_dict()
    assert step["obs"].tolist() == [[6]]
    e.set_get_interceptor(lambda v: v * 0)
    assert e["obs"].sum() == 0
    assert e.set_training(True).is_training


def test_trainable_direct_use_and_searcher_state(tmp_path):
    from ray_community_amd import tune
    from ray_community_amd.tune.schedulers import FIFOScheduler
    from ray_community_amd.tune.search import BasicVariantGenerator

    class T(tune.Trainable):
        def setup(self, config):
            self.x = config.get("x", 0)

        def step(self):
            self.x += 1
            return {"score": self.x}

        def save_checkpoint(self, d):
            return {"x": self.x}

        def load_checkpoint(self, st):
            self.x = st["x"]

        def reset_config(self, c):
            self.x = c["x"]
            return True

    t = T({"x": 1})
    r = t.train()
    assert r["score"] == 2 and r["training_iteration"] == 1 and "time_this_iter_s" in r
    ck = t.save(str(tmp_path / "ck"))
    t.train()
    t.restore(ck)
    assert t.x == 2 and t.iteration == 1
    assert t.reset({"x": 10}) and t.x == 10 and t.iteration == 0 and t.get_config() == {"x": 10}
    assert len(t.train_buffered(0.0, 3)) >= 1
    t.stop()
    s = BasicVariantGenerator()
    s._custom = 7
    s.save_to_dir(str(tmp_path), "sess")
    s2 = BasicVariantGenerator()
    s2.restore_from_dir(str(tmp_path))
    assert s2._custom == 7 and s2.set_max_concurrency(2) is False
    sch = FIFOScheduler()
    sch.save(str(tmp_path / "sch.pkl"))
    FIFOScheduler().restore(str(tmp_path / "sch.pkl"))
    assert "FIFOScheduler" in sch.debug_string()


def test_multi_agent_env_helpers_grouping_and_base_env():
    from ray_community_amd.rllib.env.base_env import convert_to_base_env
    from ray_community_amd.rllib.env.multi_agent_env import make_multi_agent

    env = make_multi_agent("CartPole-v1")({"num_agents": 2})
    ids = env.get_agent_ids()
    assert len(ids) == 2
    a = env.action_space_sample()
    assert set(a) == ids and env.action_space_contains(a)
    obs, _ = env.reset(seed=0)
    assert env.observation_space_contains(obs)
    g = env.with_agent_groups({"team": sorted(ids)})
    go, _ = g.reset(seed=0)
    assert set(go) == {"team"} and len(go["team"]) == 2
    o, r, te, tr, _ = g.step({"team": (0, 1)})
    assert isinstance(r["team"], float) and "__all__" in te
    base = convert_to_base_env(env)
    po, pr, pte, ptr, pinf, off = base.poll()
    assert set(po) == {0} and set(po[0]) == ids
    base.send_actions({0: {k: 0 for k in ids}})
    po, pr, *_ = base.poll()
    assert set(pr[0]) == ids


def test_algorithm_state_resources_and_policy_checkpoint(shutdown_only, tmp_path):
    from ray_community_amd.rllib import PPOConfig
    from ray_community_amd.rllib.algorithms.algorithm import Algorithm

    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    cfg = PPOConfig().environment("CartPole-v1").training(train_batch_size=256, model={"fcnet_hiddens": [16]})
    algo = cfg.build()
    algo.train()
    assert type(algo.get_default_config()).__name__ == "PPOConfig"
    assert algo.default_resource_request(cfg).bundles[0]["CPU"] == 1.0
    clone = Algorithm.from_state(algo.get_state())
    assert clone.iteration == 1
    w1 = algo.get_weights()
    w2 = clone.get_weights()
    assert all(np.allclose(np.asarray(w1[k]), np.asarray(w2[k])) for k in w1)
    d = algo.export_policy_checkpoint(str(tmp_path / "pol"))
    clone.import_model(d)
    with pytest.raises(NotImplementedError):
        clone.import_model("x.h5")
    assert Algorithm.merge_algorithm_configs({"m": {"a": 1, "b": 2}}, {"m": {"b": 3}}) == {"m": {"a": 1, "b": 3}}
    algo.stop()
    clone.stop()


def test_serve_deployment_properties():
    from ray_community_amd import serve

    @serve.deployment(num_replicas=2, max_ongoing_requests=7, version="v1", ray_actor_options={"num_cpus": 0.5},
                      route_prefix="/x")
    class D:
        pass

    assert D.name == "D" and D.version == "v1" and D.ray_actor_options == {"num_cpus": 0.5}
    assert D.max_concurrent_queries == 7 and D.route_prefix == "/x" and D.url.endswith("/x")
    D.set_logging_config({"log_level": "DEBUG"})
    assert D.logging_config == {"log_level": "DEBUG"}


def test_config_and_block_apis():
    import numpy as np

    from ray_community_amd import data
    from ray_community_amd.air import Result, RunConfig, ScalingConfig
    from ray_community_amd.data import aggregate as A
    from ray_community_amd.data.block import BlockAccessor
    from ray_community_amd.serve.config import AutoscalingConfig, HTTPOptions
    from ray_community_amd.serve.schema import LoggingConfig

    sc = ScalingConfig.from_placement_group_factory({"bundles": [{"CPU": 1}, {"CPU": 2, "GPU": 1}, {"CPU": 2, "GPU": 1}]})
    assert sc.num_workers == 2 and sc.use_gpu and sc.trainer_resources == {"CPU": 1}
    assert RunConfig(storage_path="/tmp/x").local_dir == "/tmp/x"
    r = Result(metrics={}, checkpoint=None, best_checkpoints=[("a", {"acc": 0.5}), ("b", {"acc": 0.9})])
    assert r.get_best_checkpoint("acc", "max") == "b" and r.get_best_checkpoint("acc", "min") == "a"
    ctx = data.DataContext.get_current()
    ctx.set_config("plugin.x", 3)
    assert ctx.get_config("plugin.x") == 3
    ctx.remove_config("plugin.x")
    assert ctx.get_config("plugin.x") is None and ctx.min_parallelism == 200
    ctx.execution_options.validate()
    ac = AutoscalingConfig(min_replicas=1, max_replicas=4, upscale_smoothing_factor=0.5)
    assert ac.get_upscaling_factor() == 0.5 and ac.get_downscaling_factor() == 1.0
    with pytest.raises(ValueError):
        AutoscalingConfig(min_replicas=3, max_replicas=2)
    assert HTTPOptions(location="NoServer").location_backfill_no_server().location == "NoServer"
    assert LoggingConfig(log_level=10).log_level == "DEBUG"
    with pytest.raises(Exception):
        LoggingConfig(encoding="XML")
    b = {"k": np.array([1, 2, 1, 3]), "v": np.array([1.0, 2.0, 3.0, 4.0])}
    acc = BlockAccessor.for_block(b)
    assert [x["k"].tolist() for x in acc.sort_and_partition([2, 3], "k")] == [[1, 1], [2], [3]]
    comb = BlockAccessor.for_block(acc.combine("k", [A.Sum("v"), A.Count()])).to_numpy()
    assert comb["sum(v)"].tolist() == [4.0, 2.0, 4.0] and comb["count()"].tolist() == [2, 1, 1]
    bld = BlockAccessor.builder()
    bld.add({"k": 9, "v": 1.0})
    bld.add_block(b)
    assert BlockAccessor(bld.build()).num_rows() == 5
    assert set(acc.zip({"w": np.arange(4)})) == {"k", "v", "w"}


def test_legacy_reader_datasource(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    from ray_community_amd.data import Datasource

    class Legacy(Datasource):
        def create_reader(self, n=10):
            class R:
                def get_read_tasks(self, parallelism):
                    return [lambda i=i: {"x": [i]} for i in range(n)]

                def estimate_inmemory_data_size(self):
                    return 8 * n
            return R()

    src = Legacy()
    assert src.should_create_reader() and src.get_name() == "Legacy"
    assert sorted(r["x"] for r in ray.data.read_datasource(src, n=5).take_all()) == [0, 1, 2, 3, 4]
