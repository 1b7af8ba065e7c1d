"""APPO target network (tau / target_update_frequency, KL against the target) and the IMPALA /
APPO learner queue (reference rllib/algorithms/appo/appo.py:109-132,265-309; learner_thread.py)."""
import pytest
import torch

import ray_community_amd as ray


def _appo(**training):
    from ray_community_amd.rllib import APPOConfig

    return (APPOConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=0, num_envs_per_env_runner=4, rollout_fragment_length=16)
            .training(lr=1e-3, train_batch_size=64, model={"fcnet_hiddens": [16]}, **training)
            .debugging(seed=3)).build()


def _info(r):
    return r["info"]["learner"]["default_policy"]


def _flat(module):
    return torch.cat([p.detach().float().reshape(-1).cpu() for p in module.parameters()])


@pytest.mark.parametrize("freq", [1, 3])
def test_appo_target_lags_online_by_target_update_frequency(shutdown_only, freq):
    ray.init(num_cpus=2)
    algo = _appo(learner_queue_size=0, target_update_frequency=freq, tau=1.0)
    lr = algo.learner_group.local
    history = [_flat(lr.module)]  # online weights after 0, 1, 2, ... updates
    for u in range(1, 8):
        r = _info(algo.train())
        history.append(_flat(lr.module))
        tgt = _flat(lr.target)
        last = (u // freq) * freq  # the target was last refreshed after update `last`
        assert torch.equal(tgt, history[last]), (u, last)
        assert r["target_updated"] == (1 if u % freq == 0 else 0)
        assert r["num_target_updates"] == u // freq
        if last < u:
            assert not torch.equal(tgt, history[u])
    algo.stop()


def test_appo_polyak_tau_and_kl_against_target(shutdown_only):
    ray.init(num_cpus=2)
    algo = _appo(learner_queue_size=0, target_update_frequency=1, tau=0.25, use_kl_loss=True, kl_coeff=0.5,
                 kl_target=1e-9)
    lr = algo.learner_group.local
    w0 = _flat(lr.module)
    algo.train()  # target created = w0, then refreshed once: 0.25 * w1 + 0.75 * w0
    w1 = _flat(lr.module)
    assert torch.allclose(_flat(lr.target), 0.25 * w1 + 0.75 * w0, atol=1e-6)
    r = _info(algo.train())
    assert r["mean_kl"] > 0  # the KL is taken against the (lagging) target policy
    # update 1: target == online, KL 0 < kl_target / 2 -> x0.5; update 2: KL >> 2 * kl_target -> x1.5
    assert r["kl_coeff"] == pytest.approx(0.5 * 0.5 * 1.5)
    # the target network and counters travel with the learner state (checkpoint / restore)
    st = lr.get_state()
    assert "target" in st and st["num_target_updates"] == 2
    algo.stop()


def test_impala_learner_queue_overlaps_sampling_and_learning(shutdown_only):
    from ray_community_amd.rllib import IMPALAConfig

    ray.init(num_cpus=4)
    algo = (IMPALAConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=2, num_envs_per_env_runner=8, rollout_fragment_length=32)
            .training(lr=1e-3, train_batch_size=256, learner_queue_size=4,
                      model={"fcnet_hiddens": [512, 512, 512]})
            .debugging(seed=1)).build()
    overlap = 0.0
    updates = []
    for _ in range(12):
        r = _info(algo.train())
        overlap = max(overlap, r["learner_overlap_s"])
        updates.append(r["num_learner_updates"])
    algo.stop()
    assert updates[-1] >= 6 and updates == sorted(updates)
    assert overlap > 0.0  # the driver kept collecting samples while the learner thread trained
    assert r["num_weight_broadcasts"] >= 2


def test_impala_inline_mode_still_available(shutdown_only):
    from ray_community_amd.rllib import IMPALAConfig

    ray.init(num_cpus=2)
    algo = (IMPALAConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=0, num_envs_per_env_runner=4, rollout_fragment_length=16)
            .training(train_batch_size=64, learner_queue_size=0, model={"fcnet_hiddens": [16]})).build()
    r = _info(algo.train())
    assert "learner_overlap_s" not in r and r["num_weight_broadcasts"] >= 1
    algo.stop()
