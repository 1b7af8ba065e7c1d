"""Conservative Q-Learning (reference: ``rllib/algorithms/cql/cql.py``, ``cql_torch_policy.py``):
offline SAC whose critics are pushed down on actions the dataset does not contain (uniform
samples and the current policy's actions, importance-corrected by their log-densities) and up on
the logged actions; the actor behaviour-clones the data for the first ``bc_iters`` updates.

Reads logged transitions (``obs, actions, rewards, new_obs, terminateds``) with
``config.offline_data(input_=...)``; evaluation runs the deterministic policy in the env.
"""
from __future__ import annotations

from typing import Dict

from .sac import SAC, SACConfig


class CQLConfig(SACConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or CQL)
        self.bc_iters = 20000
        self.temperature = 1.0
        self.num_actions = 10
        self.lagrangian = False
        self.lagrangian_thresh = 5.0
        self.min_q_weight = 5.0
        self.num_env_runners = 0
        self.num_steps_sampled_before_learning_starts = 0
        self.min_train_timesteps_per_iteration = 100
        self.evaluation_duration = 10


class CQL(SAC):
    _default_config_cls = CQLConfig

    @classmethod
    def get_default_config(cls):
        return CQLConfig()

    def setup(self, config):
        super().setup(config)
        from ..offline import JsonReader

        if not self.config.input_ or self.config.input_ == "sampler":
            raise ValueError("CQL needs offline data: config.offline_data(input_=<dir or glob>)")
        self.reader = JsonReader(self.config.input_, seed=self.config.seed)

    def training_step(self) -> Dict:
        cfg = self.config
        info: Dict = {}
        trained = 0
        while trained < max(1, cfg.min_train_timesteps_per_iteration):
            batch = self.reader.sample(cfg.train_batch_size)
            if batch.count > cfg.train_batch_size:
                batch = batch.slice(0, cfg.train_batch_size)
            info = self.learner_group.update("cql", batch)
            trained += batch.count
            self._updates += 1
        self._sync_weights()
        info["_steps_this_iter"] = 0
        info["num_agent_steps_trained"] = trained
        info["num_updates"] = self._updates
        return info
