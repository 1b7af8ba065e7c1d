"""RLlib package-level names of the reference (rllib/utils, utils/replay_buffers, env, evaluation,
offline, policy __init__ files): schedules, filters, numpy helpers, the extra replay buffers,
EnvContext, ExternalMultiAgentEnv, RemoteBaseEnv, builders, offline IO, build_policy_class."""
import os

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd.rllib.policy.sample_batch import MultiAgentBatch, SampleBatch


def test_schedules_and_helpers():
    from ray_community_amd.rllib import utils as U
    from ray_community_amd.rllib.utils.schedules import Scheduler

    lin = U.LinearSchedule(100, final_p=0.1, initial_p=1.0)
    assert lin(0) == 1.0 and abs(lin(50) - 0.55) < 1e-9 and lin(1000) == pytest.approx(0.1)
    pw = U.PiecewiseSchedule([(0, 1.0), (10, 0.5), (20, 0.0)], outside_value=0.0)
    assert pw(5) == 0.75 and pw(15) == 0.25 and pw(100) == 0.0
    assert U.ExponentialSchedule(10, initial_p=1.0, decay_rate=0.1)(10) == pytest.approx(0.1)
    assert U.PolynomialSchedule(10, final_p=0.0, power=2.0)(5) == pytest.approx(0.25)
    assert U.ConstantSchedule(3.0)(12345) == 3.0
    s = Scheduler([[0, 1e-3], [100, 1e-4]])
    assert s.update(50) == pytest.approx(5.5e-4) and s.update(1000) == pytest.approx(1e-4)

    assert U.merge_dicts({"a": {"b": 1, "c": 2}}, {"a": {"c": 3}}) == {"a": {"b": 1, "c": 3}}
    assert U.force_list(None) == [] and U.force_list(3) == [3] and U.force_tuple([1, 2]) == (1, 2)
    assert U.one_hot(np.array([0, 2]), depth=3).tolist() == [[1, 0, 0], [0, 0, 1]]
    assert np.allclose(U.softmax(np.array([0.0, 0.0])), [0.5, 0.5])
    out, (c, h) = U.lstm(np.ones((2, 3, 4)), np.zeros((4 + 5, 20)))
    assert out.shape == (2, 3, 5) and h.shape == (2, 5)
    U.check({"a": [1.0, 2.0]}, {"a": [1.0, 2.0 + 1e-7]})
    U.check(1.0, 2.0, false=True)
    with pytest.raises(AssertionError):
        U.check([1, 2], [1, 3])
    assert [fw for fw in U.framework_iterator({}, frameworks=("tf2", "torch"))] == ["torch"]
    assert U.try_import_tf() == (None, None, None)

    class Base:
        def f(self):
            return 1

    class Sub(Base):
        @U.override(Base)
        def f(self):
            return 2

    with pytest.raises(NameError):
        U.override(Base)(lambda self: 0)


def test_mean_std_filter_and_manager():
    from ray_community_amd.rllib.utils.filter import FilterManager, MeanStdFilter

    rng = np.random.default_rng(0)
    data = rng.normal(3.0, 2.0, size=(4000, 2))
    local = MeanStdFilter((2,), clip=None)
    workers = [MeanStdFilter((2,), clip=None) for _ in range(2)]
    workers[0](data[:2000])
    workers[1](data[2000:])
    new = FilterManager.synchronize({"obs": local}, [{"obs": w} for w in workers])
    assert np.allclose(local.running_stats.mean, data.mean(0), atol=1e-6)
    assert np.allclose(local.running_stats.std, data.std(0, ddof=1), atol=1e-6)
    workers[0].sync(new[0]["obs"])
    assert workers[0].buffer.n == 0 and workers[0].running_stats.n == 4000
    y = local(data[:5], update=False)
    assert np.allclose(y, (data[:5] - data.mean(0)) / data.std(0, ddof=1), atol=1e-3)


def test_extra_replay_buffers():
    from ray_community_amd.rllib.env.single_agent_episode import SingleAgentEpisode
    from ray_community_amd.rllib.utils.replay_buffers import (FifoReplayBuffer, MultiAgentMixInReplayBuffer,
                                                              MultiAgentPrioritizedReplayBuffer,
                                                              PrioritizedEpisodeReplayBuffer, ReservoirReplayBuffer)

    f = FifoReplayBuffer(8)
    f.add(SampleBatch({"x": np.arange(6)}))
    assert f.sample(4)["x"].tolist() == [0, 1, 2, 3] and len(f) == 2
    r = ReservoirReplayBuffer(50, seed=1)
    for i in range(20):
        r.add(SampleBatch({"x": np.arange(100 * i, 100 * i + 100)}))
    assert len(r) == 50 and r.num_added == 2000 and r.storage["x"][:50].max() > 1000  # late rows got in

    mp = MultiAgentPrioritizedReplayBuffer(100, prioritized_replay_alpha=1.0, seed=0)
    mp.add(MultiAgentBatch({"p": SampleBatch({"x": np.arange(10)})}, 10))
    s = mp.sample(5)
    assert "weights" in s["p"] and s["p"]["x"].shape == (5,)
    mp.update_priorities({"p": (np.arange(10), np.r_[np.zeros(9), 100.0])})
    assert (mp.sample(200)["p"]["x"] == 9).mean() > 0.9

    mix = MultiAgentMixInReplayBuffer(100, replay_ratio=0.5, seed=0)
    mix.add(SampleBatch({"x": np.arange(10)}))
    first = mix.sample()["default_policy"]
    assert first["x"].tolist()[:10] == list(range(10))
    mix.add(SampleBatch({"x": np.arange(100, 104)}))
    second = mix.sample()["default_policy"]["x"]
    assert second.shape == (8,) and set(second[:4]) == {100, 101, 102, 103}

    ep = SingleAgentEpisode()
    ep.add_env_reset(np.zeros(2))
    for t in range(10):
        ep.add_env_step(np.full(2, t + 1.0), t, float(t), terminated=t == 9)
    pb = PrioritizedEpisodeReplayBuffer(1000, alpha=1.0, seed=0)
    pb.add(ep)
    b = pb.sample(4)
    assert b["weights"].shape == (4,)
    pb.update_priorities([0.0, 0.0, 0.0, 0.0])
    drawn = pb.sample(8)
    assert drawn[SampleBatch.OBS].shape == (8, 2)


def test_env_context_reaches_the_env_creator(ray_start_regular):
    from ray_community_amd.rllib.env import EnvContext, EnvRunner, register_env
    from ray_community_amd.rllib.env.envs import CartPoleVec

    seen = []

    class _Env:
        def __init__(self, ctx):
            seen.append((type(ctx).__name__, ctx.worker_index, ctx.get("k")))
            self._v = CartPoleVec(1)
            self.observation_space, self.action_space = self._v.observation_space, \
                self._v.action_space

        def reset(self, seed=None):
            o, i = self._v.reset()
            return o[0], {}

        def step(self, a):
            o, r, te, tr, i = self._v.step(np.asarray([a]))
            return o[0], float(r[0]), bool(te[0]), bool(tr[0]), {}

    register_env("ctx_env", lambda cfg: _Env(cfg))
    EnvRunner({"env": "ctx_env", "env_config": {"k": 7}, "num_envs_per_env_runner": 1}, worker_index=3)
    assert seen and seen[0] == ("EnvContext", 3, 7)
    c = EnvContext({"a": 1}, worker_index=1).copy_with_overrides(vector_index=2)
    assert c["a"] == 1 and c.vector_index == 2 and c.worker_index == 1


def test_external_multi_agent_env_and_remote_base_env(ray_start_regular):
    from ray_community_amd.rllib.env import ExternalMultiAgentEnv, RemoteBaseEnv

    class _Sim(ExternalMultiAgentEnv):
        def run(self):
            eid = self.start_episode()
            act = self.get_action(eid, {"a": 1, "b": 2})
            self.log_returns(eid, {"a": 1.0})
            self.log_returns(eid, {"a": 0.5, "b": 2.0})
            self.result = act
            self.end_episode(eid, {"a": 3, "b": 4})

    sim = _Sim(None, None)
    base = sim.to_base_env()
    obs, rew, *_ = base.poll(timeout=10)
    (eid, o), = obs.items()
    assert o == {"a": 1, "b": 2} and rew[eid] == {}
    base.send_actions({eid: {"a": 0, "b": 1}})
    obs, rew, term, *_ = base.poll(timeout=10)
    assert term[eid] and rew[eid] == {"a": 1.5, "b": 2.0} and sim.result == {"a": 0, "b": 1}

    from ray_community_amd.rllib.env.envs import CartPoleVec

    class _One:
        def __init__(self, i):
            self.v = CartPoleVec(1, seed=i)

        def reset(self):
            o, _ = self.v.reset()
            return o[0], {}

        def step(self, a):
            o, r, te, tr, _ = self.v.step(np.asarray([a]))
            return o[0], float(r[0]), bool(te[0]), bool(tr[0]), {}

    renv = RemoteBaseEnv(lambda i: _One(i), 3)
    obs, *_ = renv.poll()
    assert sorted(k for k in obs) == [0, 1, 2]
    renv.send_actions({i: 0 for i in obs})
    obs, rew, term, trunc, infos, _ = renv.poll()
    assert sorted(k for k in obs) == [0, 1, 2] and all(rew[i] == 1.0 for i in range(3))
    renv.stop()


def test_evaluation_builders_and_metrics():
    from ray_community_amd.rllib.evaluation import (MultiAgentSampleBatchBuilder, SampleBatchBuilder,
                                                    summarize_episodes)

    b = SampleBatchBuilder()
    for t in range(3):
        b.add_values(obs=np.full(2, t), rewards=float(t))
    sb = b.build_and_reset()
    assert sb["obs"].shape == (3, 2) and b.count == 0
    mb = MultiAgentSampleBatchBuilder(clip_rewards=True)
    for t in range(4):
        mb.add_values("a0", "p0", rewards=-2.0 + t)
        mb.add_values("a1", "p1", rewards=1.0)
        mb.count_steps()
    out = mb.build_and_reset()
    assert out.env_steps() == 4 and out["p0"]["rewards"].tolist() == [-1, -1, 0, 1]
    m = summarize_episodes([(10.0, 5), (20.0, 10)])
    assert m["episode_reward_mean"] == 15.0 and m["episode_len_mean"] == 7.5


def test_offline_io_classes(ray_start_regular, tmp_path):
    from ray_community_amd.rllib.offline import (DatasetWriter, InputReader, IOContext, MixedInput,
                                                 ShuffledInput, get_offline_io_resource_bundles)

    class _Const(InputReader):
        def __init__(self, v):
            self.v = v

        def next(self):
            return SampleBatch({"x": np.full(2, self.v)})

    mixed = MixedInput({_Const(1): 0.25, (lambda ctx: _Const(2)): 0.75}, IOContext({}), seed=0)
    vals = [mixed.next()["x"][0] for _ in range(400)]
    assert 0.15 < vals.count(1) / 400 < 0.35
    with pytest.raises(ValueError):
        MixedInput({_Const(1): 0.5}, IOContext({}))
    counter = iter(range(1000))

    class _Seq(InputReader):
        def next(self):
            return SampleBatch({"x": np.asarray([next(counter)])})

    sh = ShuffledInput(_Seq(), n=8, seed=0)
    got = [int(sh.next()["x"][0]) for _ in range(30)]
    assert got != sorted(got) and len(set(got)) == 30
    w = DatasetWriter(IOContext({"output": str(tmp_path / "out"), "output_config": {"format": "json"}}),
                      max_num_samples_per_file=10)
    for i in range(3):
        w.write(SampleBatch({"obs": np.arange(5) + 5 * i, "rewards": np.ones(5, np.float32),
                             "terminateds": np.asarray([False] * 4 + [True])}))
    w.flush()
    assert os.listdir(tmp_path / "out")
    assert get_offline_io_resource_bundles({"input": "dataset", "input_config": {"parallelism": 3}}) == \
        [{"CPU": 0.5}] * 3


def test_build_policy_class_and_feature_importance():
    import torch

    from ray_community_amd.rllib.offline import FeatureImportance
    from ray_community_amd.rllib.policy import Policy, build_policy_class, build_tf_policy

    class _Model(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.zeros(3))

    def loss_fn(policy, model, dist_class, batch):
        return ((batch["obs"] @ model.w - batch["y"]) ** 2).mean()

    P = build_policy_class("LinPolicy", "torch", loss_fn=loss_fn, make_model=lambda p, o, a, c: _Model(),
                           get_default_config=lambda: {"lr": 0.1})
    p = P(None, None, {})
    x = np.random.default_rng(0).normal(size=(64, 3)).astype(np.float32)
    y = (x @ np.array([1.0, -2.0, 0.5], np.float32))
    for _ in range(300):
        stats = p.learn_on_batch({"obs": x, "y": y})
    assert stats["learner_stats"]["total_loss"] < 1e-3
    with pytest.raises(ImportError):
        build_tf_policy("X")

    class _FirstFeature(Policy):
        def compute_actions(self, obs_batch, state_batches=None, explore=True, **kw):
            return (np.asarray(obs_batch)[:, 0] > 0).astype(np.int64), [], {}

    fi = FeatureImportance(_FirstFeature(None, None), repeat=3, seed=0)
    imp = fi.estimate(SampleBatch({"obs": x}))
    assert imp["feature_0"] > 0.2 and imp["feature_1"] == 0.0 and imp["feature_2"] == 0.0


def test_rllib_metrics_helpers():
    from ray_community_amd.rllib.utils.metrics import NUM_ENV_STEPS_SAMPLED
    from ray_community_amd.rllib.utils.metrics.learner_info import LearnerInfoBuilder
    from ray_community_amd.rllib.utils.metrics.window_stat import WindowStat

    b = LearnerInfoBuilder()
    b.add_learn_on_batch_results({"learner_stats": {"loss": 1.0}, "tag": "a"})
    b.add_learn_on_batch_results({"learner_stats": {"loss": 3.0}, "tag": "b"})
    assert b.finalize() == {"default_policy": {"learner_stats": {"loss": 2.0}, "tag": "b"}}
    w = WindowStat("x", 3)
    for i in range(5):
        w.push(i)
    assert w.stats()["x_mean"] == 3.0 and w.stats()["x_count"] == 5
    assert NUM_ENV_STEPS_SAMPLED == "num_env_steps_sampled"
