"""DQN (reference: ``rllib/algorithms/dqn``): double-Q, target network, epsilon-greedy,
uniform replay."""
from __future__ import annotations

from typing import Dict

import numpy as np

from ..policy.sample_batch import SampleBatch, concat_samples
from ..utils.replay_buffers import EpisodeReplayBuffer, ReplayBuffer
from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig


class DQNConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or DQN)
        self.lr = 5e-4
        self.train_batch_size = 32
        self.replay_buffer_config = {"capacity": 50000}
        self.target_network_update_freq = 500
        self.num_steps_sampled_before_learning_starts = 1000
        self.double_q = True
        self.n_step = 1
        self.epsilon = [(0, 1.0), (10000, 0.05)]
        self.training_intensity = None
        self.rollout_fragment_length = 4
        self.td_error_loss_fn = "huber"
        self.model = {"fcnet_hiddens": [256, 256], "fcnet_activation": "relu", "vf_share_layers": True}
        # frames stacked from the episodes' observations (the episode path: replay_buffer_config
        # {"type": "EpisodeReplayBuffer"}; the module sees frame_stack x the observation)
        self.frame_stack = 1


class DQN(Algorithm):
    _default_config_cls = DQNConfig

    @classmethod
    def get_default_config(cls):
        return DQNConfig()

    def _runner_extra(self):
        extra = {"q_head": True}
        if self._episode_mode():
            extra["episode_frame_stack"] = int(getattr(self.config, "frame_stack", 1) or 1)
        return extra

    def _episode_mode(self) -> bool:
        rb = self.config.replay_buffer_config or {}
        t = rb.get("type")
        return t is EpisodeReplayBuffer or t == "EpisodeReplayBuffer"

    def setup(self, config):
        super().setup(config)
        cap = self.config.replay_buffer_config.get("capacity", 50000)
        if self._episode_mode():
            # episodes path (reference: the new API stack's DQN): runners return episode chunks,
            # the buffer samples n-step transitions with frame stacks read from the episodes
            self.buffer = EpisodeReplayBuffer(cap, seed=self.config.seed)
        else:
            self.buffer = ReplayBuffer(cap, seed=self.config.seed)
        self._last_target = 0

    def _epsilon(self):
        sched = self.config.epsilon
        t = self._timesteps_total
        for (t0, v0), (t1, v1) in zip(sched, sched[1:]):
            if t0 <= t < t1:
                return v0 + (v1 - v0) * (t - t0) / (t1 - t0)
        return sched[-1][1]

    def training_step(self) -> Dict:
        cfg = self.config
        eps = self._epsilon()
        steps = max(1, cfg.get_rollout_fragment_length()) * self.local_runner.N
        episodic = self._episode_mode()
        if episodic:
            fs = int(getattr(cfg, "frame_stack", 1) or 1)
            per_runner = self._foreach_runner("sample_episodes", steps, True, eps, fs)
            eps_list = [e for lst in per_runner for e in lst]
            self.buffer.add(eps_list)
            n = sum(len(e) for e in eps_list)
        else:
            batches = self._foreach_runner("sample_transitions", steps, eps)
            b = concat_samples(batches)
            self.buffer.add(b)
            n = b.count
        self._timesteps_total += n
        info = {"epsilon": eps}
        if self._timesteps_total >= cfg.num_steps_sampled_before_learning_starts:
            k = 1
            if cfg.training_intensity:
                k = max(1, int(round(cfg.training_intensity * n / cfg.train_batch_size)))
            for _ in range(k):
                if episodic:
                    mb = self.buffer.sample(batch_size_B=cfg.train_batch_size, n_step=int(cfg.n_step),
                                            gamma=float(cfg.gamma), frame_stack=fs)
                else:
                    mb = self.buffer.sample(cfg.train_batch_size)
                mb.pop("batch_indexes", None)
                info.update(self.learner_group.update("dqn", mb))
            if self._timesteps_total - self._last_target >= cfg.target_network_update_freq:
                self.learner_group.call("sync_target")
                self._last_target = self._timesteps_total
            self._sync_weights()
        info["_steps_this_iter"] = n
        return info


def __getattr__(name):  # old-API-stack policy names of the reference package
    from ._old_stack import policy_alias

    return policy_alias(name, __name__)
