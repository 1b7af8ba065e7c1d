"""``PolicySpec`` (reference: ``rllib/policy/policy.py``): how to build one policy of a
multi-agent setup. Spaces left as ``None`` are taken from the env agents mapped to the policy."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class PolicySpec:
    policy_class: Any = None
    observation_space: Any = None
    action_space: Any = None
    config: Optional[Dict] = field(default=None)


class Policy:
    """Old-API-stack policy interface (reference ``rllib/policy/policy.py``): action computation
    and weights. Algorithms here train RLModules through Learners; ``TorchPolicy`` wraps one so
    code written against ``compute_actions`` / ``get_weights`` keeps working."""

    def __init__(self, observation_space, action_space, config: Optional[Dict] = None):
        self.observation_space = observation_space
        self.action_space = action_space
        self.config = dict(config or {})

    def compute_actions(self, obs_batch, state_batches=None, explore: bool = True, **kw):
        raise NotImplementedError

    def compute_single_action(self, obs, state=None, explore: bool = True, **kw):
        import numpy as np

        acts, _, info = self.compute_actions(np.asarray(obs)[None], explore=explore)
        return acts[0], [], {k: v[0] for k, v in info.items()}

    def get_weights(self):
        raise NotImplementedError

    def set_weights(self, weights):
        raise NotImplementedError

    def get_state(self):
        return {"weights": self.get_weights()}

    def set_state(self, state):
        self.set_weights(state["weights"])


class TorchPolicy(Policy):
    def __init__(self, observation_space, action_space, config: Optional[Dict] = None, model=None):
        super().__init__(observation_space, action_space, config)
        if model is None:
            from ..core.rl_module import make_module

            model = make_module(self.config, observation_space, action_space)
        self.model = model

    def compute_actions(self, obs_batch, state_batches=None, explore: bool = True, **kw):
        import numpy as np
        import torch

        dev = next(self.model.parameters()).device
        obs = torch.as_tensor(np.asarray(obs_batch), device=dev)
        if explore:
            a, logp, v, logits = self.model.forward_exploration(obs)
            info = {"action_logp": logp.cpu().numpy(), "vf_preds": v.cpu().numpy(),
                    "action_dist_inputs": logits.cpu().numpy()}
        else:
            a, v = self.model.forward_inference(obs)
            info = {"vf_preds": v.cpu().numpy()}
        return a.cpu().numpy(), [], info

    def get_weights(self):
        return self.model.get_state()

    def set_weights(self, weights):
        self.model.set_state(weights)


class TFPolicy(Policy):
    def __init__(self, *a, **k):
        raise ImportError("TensorFlow is not installed: use TorchPolicy / the torch RLModules")
