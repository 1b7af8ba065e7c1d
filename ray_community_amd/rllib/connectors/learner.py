"""Learner connector pieces (reference: ``rllib/connectors/learner/
general_advantage_estimation.py`` and ``rllib/connectors/common/``). They run inside the
learner on the env-major ``[N, T]`` train batch already resident on the learner's device."""
from __future__ import annotations

import torch

from ... import ops
from .connector_v2 import ConnectorV2


class GeneralAdvantageEstimation(ConnectorV2):
    """Adds ``advantages`` and ``value_targets`` columns (GAE over the ``[N, T]`` fragments with
    the exact ``next_vf_preds`` bootstraps; the HIP kernel on GPU). The PPO loss uses the columns
    when present instead of computing GAE itself."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, gamma: float = 0.99,
                 lambda_: float = 1.0, **kw):
        self.gamma, self.lam = gamma, lambda_
        super().__init__(input_observation_space, input_action_space, **kw)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        term = batch["terminateds"]
        done = term | batch["truncateds"]
        adv, vt = ops.compute_gae(batch["rewards"], batch["vf_preds"], term, done, self.gamma, self.lam,
                                  next_values=batch["next_vf_preds"])
        batch["advantages"], batch["value_targets"] = adv, vt
        return batch


class ClipRewards(ConnectorV2):
    """Clips (``limit`` > 0) or signs (``limit`` is True) the ``rewards`` column."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, limit=1.0, **kw):
        self.limit = limit
        super().__init__(input_observation_space, input_action_space, **kw)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        r = batch["rewards"]
        batch["rewards"] = torch.sign(r) if self.limit is True else r.clamp(-float(self.limit), float(self.limit))
        return batch

# the reference package's default pieces (see connectors/common.py)
from .common import (AddColumnsFromEpisodesToTrainBatch, AddObservationsFromEpisodesToBatch, AddStatesFromEpisodesToBatch, AgentToModuleMapping, BatchIndividualItems, NumpyToTensor)  # noqa: E402,F401
from .connector_v2 import LearnerConnectorPipeline  # noqa: E402,F401
