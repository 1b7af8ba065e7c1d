"""RLlib algorithm lifecycle edge cases (reference test models: rllib/algorithms/tests/
test_algorithm.py (save / restore / from_checkpoint round trips, get/set_weights,
compute_single_action), test_algorithm_config.py (copy / freeze / to_dict))."""
import numpy as np
import pytest
import torch

import ray_community_amd as ray
from ray_community_amd.rllib.algorithms.ppo import PPOConfig


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _config():
    return (PPOConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=0, rollout_fragment_length=64)
            .training(train_batch_size=256, minibatch_size=64, num_epochs=2))


def _flat(w):
    out = []

    def walk(x):
        if isinstance(x, dict):
            for k in sorted(x):
                walk(x[k])
        elif isinstance(x, (list, tuple)):
            for v in x:
                walk(v)
        elif isinstance(x, (np.ndarray, torch.Tensor)):
            out.append(np.asarray(x.detach().cpu() if isinstance(x, torch.Tensor) else x, dtype=np.float64).ravel())

    walk(w)
    return np.concatenate(out) if out else np.zeros(0)


def test_save_restore_round_trip_preserves_weights_and_iteration(session, tmp_path):
    algo = _config().build()
    try:
        algo.train()
        algo.train()
        w = _flat(algo.get_weights())
        path = algo.save(str(tmp_path / "ckpt"))
        it = algo.iteration
    finally:
        algo.stop()
    path = getattr(path, "checkpoint", path)
    path = getattr(path, "path", path)
    algo2 = _config().build()
    try:
        algo2.restore(path)
        assert algo2.iteration == it
        assert np.allclose(_flat(algo2.get_weights()), w)
        algo2.train()                                     # training continues after restore
        assert algo2.iteration == it + 1
    finally:
        algo2.stop()


def test_set_weights_and_single_action(session):
    a, b = _config().build(), _config().build()
    try:
        a.train()
        b.set_weights(a.get_weights())
        assert np.allclose(_flat(a.get_weights()), _flat(b.get_weights()))
        obs = np.zeros(4, dtype=np.float32)
        act = a.compute_single_action(obs, explore=False)
        act = act[0] if isinstance(act, tuple) else act
        assert int(act) in (0, 1)
        act_b = b.compute_single_action(obs, explore=False)
        act_b = act_b[0] if isinstance(act_b, tuple) else act_b
        assert int(act) == int(act_b)                    # same weights, same greedy action
    finally:
        a.stop()
        b.stop()


def test_config_copy_is_independent():
    c = _config()
    d = c.copy()
    d.training(lr=0.123)
    assert c.lr != 0.123 and d.lr == 0.123
    assert c.to_dict()["train_batch_size"] == 256
