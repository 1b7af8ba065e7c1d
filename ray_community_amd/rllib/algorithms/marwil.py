"""MARWIL and BC (reference: ``rllib/algorithms/marwil/marwil.py``, ``bc/bc.py``): offline
policy learning from logged batches (``config.offline_data(input_=...)``). MARWIL weights the
log-likelihood of logged actions by exp(beta * A / ||A||) with A = discounted return - V(s)
(returns computed by the HIP GAE kernel with lambda = 1); BC is the beta = 0 special case."""
from __future__ import annotations

from typing import Dict

from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig


class MARWILConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or MARWIL)
        self.beta = 1.0
        self.vf_coeff = 1.0
        self.moving_average_sqd_adv_norm_update_rate = 1e-8
        self.moving_average_sqd_adv_norm_start = 100.0
        self.lr = 1e-4
        self.train_batch_size = 2000
        self.num_env_runners = 0
        self.evaluation_duration = 10


class MARWIL(Algorithm):
    _default_config_cls = MARWILConfig

    @classmethod
    def get_default_config(cls):
        return cls._default_config_cls()

    def setup(self, config):
        super().setup(config)
        from ..offline import DatasetReader, JsonReader, get_dataset_and_shards

        if not self.config.input_ or self.config.input_ == "sampler":
            raise ValueError("MARWIL/BC need offline data: config.offline_data(input_=<dir or glob> | \"dataset\")")
        if self.config.input_ == "dataset":  # Ray Data rows (reference DatasetReader)
            ds, _ = get_dataset_and_shards(self.config)
            self.reader = DatasetReader(ds, batch_size=min(self.config.train_batch_size, 4096),
                                        gamma=self.config.gamma, seed=self.config.seed)
        else:
            self.reader = JsonReader(self.config.input_, seed=self.config.seed)

    def training_step(self) -> Dict:
        batch = self.reader.sample(self.config.train_batch_size)
        info = self.learner_group.update("marwil", batch)
        info["_steps_this_iter"] = 0
        info["num_agent_steps_trained"] = batch.count
        return info


class BCConfig(MARWILConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or BC)
        self.beta = 0.0
        self.vf_coeff = 0.0


class BC(MARWIL):
    _default_config_cls = BCConfig
