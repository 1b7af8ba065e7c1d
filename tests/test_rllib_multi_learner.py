"""8-learner rehearsal on CPU (gloo world 8): the BASELINE "PPO, 8 GPU learners" config's learner
group takes exactly the single-learner trajectory (reference rllib/core/learner/learner_group.py;
DDP over the learners' process group, group-wide advantage statistics), and reports per-rank
update times and exposed all-reduce time."""
import torch

import ray_community_amd as ray
from ray_community_amd.rllib import PPOConfig


def test_eight_learners_match_one_learner_over_three_updates(shutdown_only):
    from ray_community_amd.rllib.core.learner import LearnerGroup
    from ray_community_amd.rllib.env.env_runner import EnvRunner

    ray.init(num_cpus=8)
    cfg = (PPOConfig().environment("CartPole-v1").env_runners(num_envs_per_env_runner=8)
           .training(lr=1e-3, train_batch_size=512, minibatch_size=512, num_epochs=1, use_kl_loss=False,
                     model={"fcnet_hiddens": [32, 32]}).debugging(seed=5))
    cfg.adam_epsilon = 1e-3  # smooth first Adam steps: fp32 summation-order noise stays tiny
    runner = EnvRunner(cfg.runner_dict(), 0)
    batches = [runner.sample(512) for _ in range(3)]
    obs_sp, act_sp = runner.spaces()
    d1 = cfg.to_dict()
    one = LearnerGroup(d1, obs_sp, act_sp)
    eight = LearnerGroup(dict(d1, num_learners=8), obs_sp, act_sp)
    try:
        w0 = {k: v.clone() for k, v in one.get_weights().items()}
        assert all(torch.equal(w0[k], eight.get_weights()[k]) for k in w0)
        for i, b in enumerate(batches):
            s1 = one.update("ppo", b)
            s8 = eight.update("ppo", b)
            assert abs(s1["policy_loss"] - s8["policy_loss"]) < 1e-4, i
            assert len(s8["rank_update_time_s"]) == 8 and all(t > 0 for t in s8["rank_update_time_s"])
            assert len(s8["rank_exposed_comm_ms"]) == 8 and s8["exposed_comm_ms"] >= 0.0
        wa, wb = one.get_weights(), eight.get_weights()
        for k in wa:
            assert not torch.equal(wa[k], w0[k]) or k.endswith("bias"), k
            assert torch.allclose(wa[k], wb[k], atol=1e-5, rtol=1e-4), (k, (wa[k] - wb[k]).abs().max())
        # every learner holds the same replica
        reps = ray.get([w.call.remote("get_weights") for w in eight.wg.workers])
        for r in reps[1:]:
            assert all(torch.equal(r[k], reps[0][k]) for k in r)
    finally:
        eight.shutdown()


def test_synthetic_atari_packed_frame_stack_is_bitwise_equal():
    """The packed uint32 frame-stack render (one in-place shift per step) produces exactly the
    observations, rewards, terminations and final observations of the per-channel HWC render."""
    import numpy as np

    from ray_community_amd.rllib.env.envs import SyntheticAtariVec

    a = SyntheticAtariVec(num_envs=8, seed=11, max_episode_steps=120)
    b = SyntheticAtariVec(num_envs=8, seed=11, max_episode_steps=120)
    b._packed = None  # the generic path
    assert a._packed is not None
    oa, _ = a.reset()
    ob, _ = b.reset()
    assert np.array_equal(oa, ob)
    rng = np.random.default_rng(5)
    resets = 0
    for _ in range(1500):
        act = rng.integers(0, 6, 8)
        ra, rb = a.step(act), b.step(act)
        for x, y in zip(ra[:4], rb[:4]):
            assert np.array_equal(x, y)
        assert np.array_equal(ra[4]["final_obs"], rb[4]["final_obs"])
        resets += int((ra[2] | ra[3]).sum())
    assert resets > 0


def test_ppo_fragment_refs_to_learner_actor_match_materialised_path(shutdown_only, monkeypatch):
    """PPO with a learner actor takes the runners' fragments by reference (the learner maps them
    from the shared-memory store and copies each to its device as it arrives); the weights after
    three iterations are bitwise those of the path that materialises them in the driver."""
    import torch

    from ray_community_amd.rllib.algorithms import algorithm as A

    ray.init(num_cpus=6)

    def run():
        cfg = (PPOConfig().environment("CartPole-v1").env_runners(num_env_runners=2, num_envs_per_env_runner=4)
               .training(lr=1e-3, train_batch_size=256, minibatch_size=128, num_epochs=2,
                         model={"fcnet_hiddens": [16]})
               .learners(num_learners=1).debugging(seed=7))
        algo = cfg.build()
        try:
            steps = [algo.train()["num_env_steps_sampled_this_iter"] for _ in range(3)]
            return algo.learner_group.get_weights(), steps
        finally:
            algo.stop()

    w_refs, s_refs = run()
    monkeypatch.setenv("RCA_RLLIB_FRAGMENT_REFS", "0")
    w_mat, s_mat = run()
    assert s_refs == s_mat == [256, 256, 256]
    assert all(torch.equal(w_refs[k], w_mat[k]) for k in w_refs)
