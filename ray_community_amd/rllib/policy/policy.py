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


def build_policy_class(name: str, framework: str = "torch", *, loss_fn=None, get_default_config=None,
                       optimizer_fn=None, stats_fn=None, make_model=None, mixins=None, **kw):
    """A ``TorchPolicy`` subclass named ``name`` (reference rllib/policy/policy_template.py):
    ``loss_fn(policy, model, dist_class, train_batch) -> loss`` drives ``learn_on_batch`` with the
    optimizer from ``optimizer_fn(policy, config)`` (Adam at ``config["lr"]`` by default)."""
    if framework != "torch":
        raise ImportError(f"framework={framework!r} is not installed here; only torch policies can be built")

    def _init(self, observation_space, action_space, config=None):
        cfg = dict(get_default_config() if get_default_config else {})
        cfg.update(config or {})
        model = make_model(self, observation_space, action_space, cfg) if make_model else None
        TorchPolicy.__init__(self, observation_space, action_space, cfg, model=model)
        import torch

        self._optimizer = optimizer_fn(self, self.config) if optimizer_fn else \
            torch.optim.Adam(self.model.parameters(), lr=float(self.config.get("lr", 1e-3)))

    def learn_on_batch(self, samples):
        import torch

        if loss_fn is None:
            raise NotImplementedError(f"{name} was built without a loss_fn")
        dev = next(self.model.parameters()).device
        batch = {k: torch.as_tensor(v, device=dev) for k, v in samples.items()}
        loss = loss_fn(self, self.model, None, batch)
        self._optimizer.zero_grad()
        loss.backward()
        self._optimizer.step()
        stats = stats_fn(self, batch) if stats_fn else {}
        return {"learner_stats": dict(stats, total_loss=float(loss.detach()))}

    bases = tuple(mixins or ()) + (TorchPolicy,)
    return type(name, bases, {"__init__": _init, "learn_on_batch": learn_on_batch})


def build_tf_policy(*a, **k):
    raise ImportError("TensorFlow is not installed: use build_policy_class(..., framework='torch')")
