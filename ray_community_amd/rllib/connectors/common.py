"""The reference's default connector pieces (rllib/connectors/common/*,
env_to_module/*, module_to_env/*, learner/*) for user-assembled pipelines.

This framework's env runner is vectorised: it builds the module's batch for all N sub-envs in
one go (observations, recurrent states, batching, host->device copies, action sampling and the
hand-off back to the env happen in the runner itself; see connector_v2.py). The default pieces
are therefore thin here -- each does its one transformation when the batch still needs it
(list items to stack, numpy to tensors, tensors to numpy, a singleton time axis to drop,
actions to sample from distribution inputs) and passes the batch through otherwise -- so a
pipeline written as the reference's default one (``[AddObservationsFromEpisodesToBatch(),
BatchIndividualItems(), NumpyToTensor(), ...]``) runs unchanged."""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np

from .connector_v2 import ConnectorV2


def _episodes_list(episodes):
    return episodes if isinstance(episodes, (list, tuple)) else None


class AddObservationsFromEpisodesToBatch(ConnectorV2):
    """``batch["obs"]`` from the episodes' latest observations when the batch lacks it."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        eps = _episodes_list(episodes)
        if "obs" not in batch and eps:
            batch["obs"] = [e.get_observations(-1) for e in eps]
        return batch


class AddStatesFromEpisodesToBatch(ConnectorV2):
    """Recurrent states live in the runner (one row per sub-env); nothing to add here."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        return batch


class AddColumnsFromEpisodesToTrainBatch(ConnectorV2):
    """Train-batch columns from episodes (obs / actions / rewards / terminateds) when the
    learner receives episodes instead of a built batch."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        eps = _episodes_list(episodes)
        if eps and "obs" not in batch:
            from ..policy.sample_batch import concat_samples

            b = concat_samples([e.to_sample_batch() for e in eps])
            for k, v in b.items():
                batch.setdefault(k, v)
        return batch


class AgentToModuleMapping(ConnectorV2):
    """Per-agent batches -> per-module batches (the multi-agent runner groups by module already)."""

    def __init__(self, *args, module_specs=None, agent_to_module_mapping_fn=None, **kw):
        super().__init__(*args, **kw)
        self.agent_to_module_mapping_fn = agent_to_module_mapping_fn

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        return batch


class ModuleToAgentUnmapping(AgentToModuleMapping):
    pass


class BatchIndividualItems(ConnectorV2):
    """Lists of per-env items -> one stacked array per column."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        for k, v in list(batch.items()):
            if isinstance(v, list) and v and not isinstance(v[0], (str, bytes, dict)):
                batch[k] = np.stack([np.asarray(x) for x in v])
        return batch


class UnBatchToIndividualItems(ConnectorV2):
    """The vectorised env consumes the batched actions as they are."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        return batch


class ListifyDataForVectorEnv(UnBatchToIndividualItems):
    pass


class NumpyToTensor(ConnectorV2):
    """numpy columns -> torch tensors on the module's device (or ``device``)."""

    def __init__(self, *args, device=None, pin_memory: bool = False, **kw):
        super().__init__(*args, **kw)
        self.device = device

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        import torch

        dev = self.device
        if dev is None and rl_module is not None:
            p = next(iter(rl_module.parameters()), None) if hasattr(rl_module, "parameters") else None
            dev = p.device if p is not None else None
        for k, v in list(batch.items()):
            if isinstance(v, np.ndarray) and v.dtype != object:
                batch[k] = torch.as_tensor(v, device=dev)
        return batch


class TensorToNumpy(ConnectorV2):
    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        for k, v in list(batch.items()):
            if hasattr(v, "detach"):
                batch[k] = v.detach().cpu().numpy()
        return batch


class RemoveSingleTsTimeRankFromBatch(ConnectorV2):
    """Drop a singleton time axis ([B, 1, ...] -> [B, ...]) left by a recurrent forward."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        for k, v in list(batch.items()):
            shape = getattr(v, "shape", None)
            if shape is not None and len(shape) >= 2 and shape[1] == 1:
                batch[k] = v[:, 0]
        return batch


class GetActions(ConnectorV2):
    """Actions from ``action_dist_inputs`` when the module returned only distribution inputs:
    a sample when exploring, the distribution's deterministic action otherwise, plus logp."""

    def __call__(self, *, rl_module=None, batch, episodes=None, explore: Optional[bool] = None, **kw):
        if "actions" in batch or "action_dist_inputs" not in batch or rl_module is None:
            return batch
        import torch

        logits = batch["action_dist_inputs"]
        logits = logits if torch.is_tensor(logits) else torch.as_tensor(np.asarray(logits))
        dist = rl_module.dist(logits) if hasattr(rl_module, "dist") else rl_module.dist_cls(logits)
        a = dist.sample() if explore or explore is None else dist.deterministic_sample()
        batch["actions"] = a
        batch["action_logp"] = dist.logp(a)
        return batch


class WriteObservationsToEpisodes(ConnectorV2):
    """Connector outputs written back into episode objects (the vectorised runner records the
    transformed observations in its own buffers)."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        return batch


class AddTimeDimToBatchAndZeroPad(ConnectorV2):
    """[B, ...] -> [B, 1, ...] for modules that expect a time rank (recurrent ones chunk the
    train batch by ``max_seq_len`` in the learner instead)."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        for k, v in list(batch.items()):
            if hasattr(v, "shape") and len(v.shape) >= 1 and k in ("obs",):
                batch[k] = v[:, None]
        return batch


__all__ = ["AddObservationsFromEpisodesToBatch", "AddStatesFromEpisodesToBatch", "AddColumnsFromEpisodesToTrainBatch",
           "AgentToModuleMapping", "ModuleToAgentUnmapping", "BatchIndividualItems", "UnBatchToIndividualItems",
           "ListifyDataForVectorEnv", "NumpyToTensor", "TensorToNumpy", "RemoveSingleTsTimeRankFromBatch",
           "GetActions", "WriteObservationsToEpisodes", "AddTimeDimToBatchAndZeroPad"]
