"""IMPALA and APPO (reference: ``rllib/algorithms/impala/impala.py``, ``vtrace_torch.py``,
``rllib/algorithms/appo/appo.py``).

Asynchronous actor-learner architecture: every env runner keeps
``max_requests_in_flight_per_env_runner`` sample requests queued; each ``training_step`` takes
whichever fragments are ready (``wait``), immediately re-queues those runners, and trains on the
concatenated ``[N, T]`` fragments. Runners therefore act with weights that lag the learner by a
few updates; V-trace (a HIP kernel over the env-major fragments, ``ops.vtrace``) corrects for the
policy lag. Weights are broadcast without blocking every ``broadcast_interval`` updates (actor
calls are ordered per caller, so a runner's next fragment uses them).
"""
from __future__ import annotations

from typing import Dict, List

from ..policy.sample_batch import concat_samples
from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig


class IMPALAConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or IMPALA)
        self.vtrace = True
        self.vtrace_clip_rho_threshold = 1.0
        self.vtrace_clip_c_threshold = 1.0
        self.vtrace_clip_pg_rho_threshold = 1.0
        self.lr = 0.0005
        self.train_batch_size = 500
        self.rollout_fragment_length = 50
        self.vf_loss_coeff = 0.5
        self.entropy_coeff = 0.01
        self.grad_clip = 40.0
        self.broadcast_interval = 1
        self.max_requests_in_flight_per_env_runner = 2
        self.num_epochs = 1
        self.minibatch_size = None


class IMPALA(Algorithm):
    _default_config_cls = IMPALAConfig
    _update_kind = "impala"

    @classmethod
    def get_default_config(cls):
        return cls._default_config_cls()

    def _sample_async(self, steps: int):
        from ..._private.worker import get, wait

        cfg = self.config
        g = self.env_runner_group
        frag = cfg.get_rollout_fragment_length() * max(1, cfg.num_envs_per_env_runner)
        if not hasattr(self, "_inflight"):
            self._inflight = {}  # sample ref -> runner id
        # top every healthy runner (new, or restored by restore_workers) up to its request budget
        actors = g.manager.actors()
        per = max(1, cfg.max_requests_in_flight_per_env_runner)
        for i in g.healthy_env_runner_ids():
            for _ in range(per - sum(1 for v in self._inflight.values() if v == i)):
                self._inflight[actors[i].sample.remote(frag)] = i
        got: List = []
        n = 0
        while n < steps:
            if not self._inflight:  # no healthy remote runner left: the local one samples
                b = self.local_runner.sample(max(steps - n, self.local_runner.N))
                got.append(b)
                n += b.count
                break
            ready, _ = wait(list(self._inflight), num_returns=1)
            for ref in ready:
                i = self._inflight.pop(ref)
                try:
                    b = get(ref)
                except Exception as e:  # noqa  (the group's policy decides: raise, or drop the runner)
                    g.mark_failed(i, e)
                    for other in [r for r, j in self._inflight.items() if j == i]:
                        self._inflight.pop(other, None)
                    continue
                got.append(b)
                n += b.count
                if g.manager.is_actor_healthy(i):
                    self._inflight[g.manager.actors()[i].sample.remote(frag)] = i
        return concat_samples(got)

    def _broadcast_async(self):
        from ..._private.worker import put

        st = self.learner_group.get_weights()
        self._weights_version += 1
        self.local_runner.set_weights(st, self._weights_version)
        if self.remote_runners:
            ref = put(st)
            for r in self.remote_runners:
                r.set_weights.remote(ref, self._weights_version)

    def training_step(self) -> Dict:
        cfg = self.config
        batch = self._sample_async(cfg.train_batch_size)
        n = batch.count
        self._timesteps_total += n
        info = self.learner_group.update(self._update_kind, batch)
        self._num_updates = getattr(self, "_num_updates", 0) + 1
        if self._num_updates % max(1, cfg.broadcast_interval) == 0:
            self._broadcast_async()
        info["_steps_this_iter"] = n
        info["num_weight_broadcasts"] = self._weights_version
        return info

    def stop(self):
        self._inflight = {}
        super().stop()

    cleanup = stop


class APPOConfig(IMPALAConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or APPO)
        self.clip_param = 0.4
        self.use_kl_loss = False
        self.kl_coeff = 1.0
        self.kl_target = 0.01
        self.num_epochs = 1
        self.lr = 0.0005


class APPO(IMPALA):
    _default_config_cls = APPOConfig
    _update_kind = "appo"
