"""Soft Actor-Critic (reference: ``rllib/algorithms/sac/sac.py``): off-policy, uniform replay,
uniformly random actions until ``num_steps_sampled_before_learning_starts``, then the stochastic
tanh-Gaussian policy; ``training_intensity`` learner updates per sampled env step."""
from __future__ import annotations

from typing import Dict

from ..policy.sample_batch import concat_samples
from ..utils.replay_buffers import ReplayBuffer
from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig


class SACConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or SAC)
        self.lr = 3e-4
        self.gamma = 0.99
        self.tau = 5e-3
        self.initial_alpha = 1.0
        self.target_entropy = "auto"
        self.n_step = 1
        self.train_batch_size = 256
        self.replay_buffer_config = {"capacity": 100000}
        self.num_steps_sampled_before_learning_starts = 1500
        self.training_intensity = 1.0
        self.rollout_fragment_length = 1
        self.optimization_config = {"actor_learning_rate": 3e-4, "critic_learning_rate": 3e-4,
                                    "entropy_learning_rate": 3e-4}
        self.model = {"fcnet_hiddens": [256, 256], "fcnet_activation": "relu"}
        self.grad_clip = None


class SAC(Algorithm):
    _default_config_cls = SACConfig

    @classmethod
    def get_default_config(cls):
        return SACConfig()

    def _runner_extra(self):
        return {"module_class": "sac", "model": {**self.config.model,
                                                  "initial_alpha": self.config.initial_alpha}}

    def setup(self, config):
        super().setup(config)
        self.buffer = ReplayBuffer(self.config.replay_buffer_config.get("capacity", 100000), seed=self.config.seed)
        self._updates = 0

    def training_step(self) -> Dict:
        from ..._private.worker import get

        cfg = self.config
        warm = self._timesteps_total < cfg.num_steps_sampled_before_learning_starts
        eps = 1.0 if warm else 0.0
        steps = max(1, cfg.get_rollout_fragment_length()) * self.local_runner.N
        batches = self._foreach_runner("sample_transitions", steps, eps)
        b = concat_samples(batches)
        self.buffer.add(b)
        n = b.count
        self._timesteps_total += n
        info: Dict = {}
        if not warm:
            k = max(1, int(round(cfg.training_intensity * n)))
            for _ in range(k):
                mb = self.buffer.sample(cfg.train_batch_size)
                mb.pop("batch_indexes", None)
                info = self.learner_group.update("sac", mb)
                self._updates += 1
            self._sync_weights()
        info["_steps_this_iter"] = n
        info["num_updates"] = self._updates
        return info


def __getattr__(name):  # old-API-stack policy names of the reference package
    from ._old_stack import policy_alias

    return policy_alias(name, __name__)
