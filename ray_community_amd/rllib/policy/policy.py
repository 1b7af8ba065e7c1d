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
        return {"weights": self.get_weights(), "policy_class": type(self), "observation_space":
                self.observation_space, "action_space": self.action_space, "config": self.config}

    def set_state(self, state):
        self.set_weights(state["weights"])

    # ------------------------------------------------------------------ old-API-stack surface
    # (reference rllib/policy/policy.py; training runs through Learners here, so the methods
    # that only made sense for the old training loop delegate to learn_on_batch / compute_gradients)
    @classmethod
    def from_state(cls, state):
        klass = state["policy_class"]
        args = (state["observation_space"], state["action_space"], state.get("config"))
        pol = klass(*args, model=state["model"]) if state.get("model") is not None else klass(*args)
        pol.set_state(state)
        return pol

    def export_checkpoint(self, export_dir: str, **kw) -> None:
        import os

        import cloudpickle

        os.makedirs(export_dir, exist_ok=True)
        with open(os.path.join(export_dir, "policy_state.pkl"), "wb") as f:
            cloudpickle.dump(self.get_state(), f)

    @staticmethod
    def from_checkpoint(checkpoint, policy_ids=None):
        import os
        import pickle

        path = getattr(checkpoint, "path", checkpoint)
        with open(os.path.join(path, "policy_state.pkl"), "rb") as f:  # written by export_checkpoint
            return Policy.from_state(pickle.load(f))

    def export_model(self, export_dir: str, onnx=None) -> None:
        import os

        import torch

        if onnx:
            raise NotImplementedError("ONNX export needs the onnx package, which is not installed")
        os.makedirs(export_dir, exist_ok=True)
        model = getattr(self, "model", None)
        torch.save(model.state_dict() if model is not None else self.get_weights(),
                   os.path.join(export_dir, "model.pt"))

    def import_model_from_h5(self, import_file: str):
        raise NotImplementedError("h5 (Keras) models need TensorFlow, which is not installed")

    def make_rl_module(self):
        return getattr(self, "model", None)

    def init_view_requirements(self) -> None:
        self.view_requirements = {"obs": None, "actions": None, "rewards": None}

    def get_connector_metrics(self):
        return {}

    def reset_connectors(self, env_id) -> None:
        pass

    def restore_connectors(self, state) -> None:
        pass

    def compute_actions_from_input_dict(self, input_dict, explore: bool = True, timestep=None, **kw):
        return self.compute_actions(input_dict["obs"], explore=explore, **kw)

    def compute_log_likelihoods(self, actions, obs_batch, state_batches=None, **kw):
        raise NotImplementedError

    def postprocess_trajectory(self, sample_batch, other_agent_batches=None, episode=None):
        return sample_batch

    def loss(self, model, dist_class, train_batch):
        raise NotImplementedError

    def learn_on_batch(self, samples):
        raise NotImplementedError("this policy has no loss; see build_policy_class or the algorithms' Learners")

    def learn_on_batch_from_replay_buffer(self, replay_actor, policy_id):
        from ... import get

        batch = get(replay_actor.replay.remote(policy_id=policy_id))
        return None if batch is None else self.learn_on_batch(batch)

    def load_batch_into_buffer(self, batch, buffer_index: int = 0) -> int:
        self._loaded = getattr(self, "_loaded", {})
        self._loaded[buffer_index] = batch
        return len(batch)

    def get_num_samples_loaded_into_buffer(self, buffer_index: int = 0) -> int:
        b = getattr(self, "_loaded", {}).get(buffer_index)
        return 0 if b is None else len(b)

    def learn_on_loaded_batch(self, offset: int = 0, buffer_index: int = 0):
        b = self._loaded[buffer_index]
        mb = int(self.config.get("minibatch_size") or self.config.get("sgd_minibatch_size") or len(b))
        return self.learn_on_batch(b.slice(offset, offset + mb) if hasattr(b, "slice") else b)

    def compute_gradients(self, postprocessed_batch):
        raise NotImplementedError

    def apply_gradients(self, gradients) -> None:
        raise NotImplementedError

    def get_exploration_state(self):
        return {}

    def is_recurrent(self) -> bool:
        return bool(getattr(getattr(self, "model", None), "is_stateful", False))

    def num_state_tensors(self) -> int:
        return 2 if self.is_recurrent() else 0

    def get_initial_state(self):
        model = getattr(self, "model", None)
        if self.is_recurrent():
            h, c = model.get_initial_state(1)
            return [h[0].cpu().numpy(), c[0].cpu().numpy()]
        return []

    def apply(self, func, *args, **kwargs):
        return func(self, *args, **kwargs)

    def on_global_var_update(self, global_vars) -> None:
        self.global_timestep = int(global_vars.get("timestep", 0))

    def get_session(self):
        return None

    def get_host(self) -> str:
        import socket

        return socket.gethostname()

    def maybe_add_time_dimension(self, input_dict, seq_lens=None, framework: str = "torch"):
        return input_dict

    def maybe_remove_time_dimension(self, input_dict):
        return input_dict


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

    def get_state(self):
        st = super().get_state()
        st["model"] = self.model  # the module itself, so from_state rebuilds custom / SAC modules too
        return st

    def compute_log_likelihoods(self, actions, obs_batch, state_batches=None, **kw):
        import numpy as np
        import torch

        dev = next(self.model.parameters()).device
        with torch.no_grad():
            logits, _ = self.model.forward(torch.as_tensor(np.asarray(obs_batch), device=dev))
            return self.model.dist(logits).logp(torch.as_tensor(np.asarray(actions), device=dev)).cpu().numpy()

    def _opt(self):
        import torch

        if getattr(self, "_optimizer", None) is None:
            self._optimizer = torch.optim.Adam(self.model.parameters(), lr=float(self.config.get("lr", 1e-3)))
        return self._optimizer

    def compute_gradients(self, postprocessed_batch):
        """Gradients of ``self.loss`` on the batch: (list of numpy grads, info)."""
        import torch

        dev = next(self.model.parameters()).device
        batch = {k: torch.as_tensor(v, device=dev) for k, v in postprocessed_batch.items()}
        self._opt().zero_grad(set_to_none=True)
        loss = self.loss(self.model, getattr(self.model, "dist_cls", None), batch)
        loss.backward()
        grads = [None if p.grad is None else p.grad.detach().cpu().numpy() for p in self.model.parameters()]
        return grads, {"learner_stats": {"total_loss": float(loss.detach())}}

    def apply_gradients(self, gradients) -> None:
        import torch

        for p, g in zip(self.model.parameters(), gradients):
            p.grad = None if g is None else torch.as_tensor(g, device=p.device)
        self._opt().step()


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
