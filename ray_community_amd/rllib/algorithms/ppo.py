"""PPO (reference: ``rllib/algorithms/ppo/ppo.py``, ``ppo_torch_learner.py``)."""
from __future__ import annotations

import time

from typing import Dict

from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig


class PPOConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or PPO)
        self.lr = 5e-5
        self.lambda_ = 1.0
        self.use_gae = True
        self.use_critic = True
        self.kl_coeff = 0.2
        self.kl_target = 0.01
        self.use_kl_loss = True
        self.clip_param = 0.3
        self.vf_clip_param = 10.0
        self.vf_loss_coeff = 1.0
        self.entropy_coeff = 0.0
        self.train_batch_size = 4000
        self.minibatch_size = 128
        self.num_epochs = 30
        self.grad_clip = None

    def validate(self) -> None:
        super().validate()
        if self.minibatch_size is not None and int(self.minibatch_size) > int(self.train_batch_size):
            raise ValueError(f"minibatch_size ({self.minibatch_size}) must be <= train_batch_size "
                             f"({self.train_batch_size})")
        if int(self.num_epochs) < 1:
            raise ValueError(f"num_epochs must be >= 1, got {self.num_epochs}")
        if float(self.entropy_coeff) < 0:
            raise ValueError(f"entropy_coeff must be >= 0, got {self.entropy_coeff}")
        if float(self.clip_param) <= 0 or float(self.vf_clip_param) <= 0:
            raise ValueError("clip_param and vf_clip_param must be > 0")
        if float(self.kl_coeff) < 0:
            raise ValueError(f"kl_coeff must be >= 0, got {self.kl_coeff}")

    @property
    def sgd_minibatch_size(self):
        return self.minibatch_size

    @property
    def num_sgd_iter(self):
        return self.num_epochs


class PPO(Algorithm):
    _default_config_cls = PPOConfig
    _supports_lstm = True

    @classmethod
    def get_default_config(cls):
        return PPOConfig()

    def training_step(self) -> Dict:
        cfg = self.config
        t0 = time.perf_counter()
        if self.multi_agent:
            batch = self._sample(cfg.train_batch_size)
            n = batch.count
            t1 = time.perf_counter()
            info = {p: self.learner_groups[p].update("ppo", batch.policy_batches[p])
                    for p in self.policies_to_train if p in batch.policy_batches}
        else:
            # runner fragments go to the learner(s) as they are: stacked on the GPU, not the host.
            # With learner actors the driver does not even materialise them: the learners read
            # the runners' fragments straight from the shared-memory store (object refs)
            refs = self._sample_fragment_refs(cfg.train_batch_size, wait_ready=False)
            if refs is not None:
                frags, n = refs
            else:
                frags = self._sample_fragments(cfg.train_batch_size)
                n = sum(f.count for f in frags)
            t1 = time.perf_counter()
            info = self.learner_group.update("ppo", frags)
        t2 = time.perf_counter()
        self._timesteps_total += n
        self._sync_weights()
        t3 = time.perf_counter()
        # driver-side phase times of the iteration (sampling includes the fragments' transfer to
        # the driver; the learner phase includes the host->device copy)
        # (with fragment refs the sample phase only issues the requests: the learner phase then
        # includes waiting for the runners, overlapped with the fragments' device copies)
        phases = {"sample_time_s": t1 - t0, "learn_time_s": t2 - t1, "sync_weights_time_s": t3 - t2}
        if self.multi_agent:  # info is keyed by policy id: the iteration's phases go in each
            for v in info.values():
                v.update(phases)
        else:
            info.update(phases)
        info["_steps_this_iter"] = n
        return info


def __getattr__(name):  # old-API-stack policy names (rllib/algorithms/ppo/__init__.py)
    from ._old_stack import policy_alias

    return policy_alias(name, __name__)
