"""Module -> env connector pieces (reference: ``rllib/connectors/module_to_env/
normalize_and_clip_actions.py``). They rewrite ``batch["actions_for_env"]`` (what the env steps
with); ``batch["actions"]`` keeps the sampled actions the loss and log-probs refer to."""
from __future__ import annotations

import numpy as np

from ..utils.spaces import Box
from .connector_v2 import ConnectorV2


class NormalizeAndClipActions(ConnectorV2):
    """``normalize_actions``: the module acts in [-1, 1] and actions are unsquashed to the Box
    bounds; ``clip_actions``: actions are clipped to the bounds."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, normalize_actions: bool = True,
                 clip_actions: bool = False, **kw):
        self.normalize, self.clip = normalize_actions, clip_actions
        super().__init__(input_observation_space, input_action_space, **kw)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        s = self._input_action_space
        if not isinstance(s, Box):
            return batch
        a = np.asarray(batch["actions_for_env"], dtype=np.float32)
        lo, hi = s.low.astype(np.float32), s.high.astype(np.float32)
        if self.normalize:
            a = lo + (np.clip(a, -1.0, 1.0) + 1.0) * 0.5 * (hi - lo)
        if self.clip:
            a = np.clip(a, lo, hi)
        batch["actions_for_env"] = a
        return batch


class ClipActions(NormalizeAndClipActions):
    def __init__(self, input_observation_space=None, input_action_space=None, **kw):
        super().__init__(input_observation_space, input_action_space, normalize_actions=False, clip_actions=True)

# the reference package's default pieces (see connectors/common.py)
from .common import (GetActions, ListifyDataForVectorEnv, ModuleToAgentUnmapping, RemoveSingleTsTimeRankFromBatch, TensorToNumpy, UnBatchToIndividualItems)  # noqa: E402,F401
from .connector_v2 import ModuleToEnvPipeline  # noqa: E402,F401
