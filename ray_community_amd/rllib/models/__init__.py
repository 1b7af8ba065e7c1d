"""Old-API-stack model catalog (reference: rllib/models/{catalog,modelv2,action_dist,
preprocessors}.py, models/torch/{torch_modelv2,fcnet,torch_action_dist}.py).

New-stack training here runs on RLModules (rllib/core/rl_module.py); these classes keep code
written against ``ModelCatalog`` / ``ModelV2`` / custom models working: ``get_model_v2`` builds
a registered custom ``TorchModelV2`` or the built-in fully connected one, ``get_action_dist``
maps an action space to the torch distribution classes the RLModules use, and the preprocessors
flatten / one-hot observations."""
from __future__ import annotations

import copy
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from ..core.rl_module import Categorical, DiagGaussian, _mlp
from ..utils.spaces import Box, Dict as DictSpace, Discrete, Tuple as TupleSpace

MODEL_DEFAULTS: Dict[str, Any] = {
    "fcnet_hiddens": [256, 256],
    "fcnet_activation": "tanh",
    "conv_filters": None,
    "conv_activation": "relu",
    "post_fcnet_hiddens": [],
    "post_fcnet_activation": "relu",
    "free_log_std": False,
    "no_final_linear": False,
    "vf_share_layers": False,
    "use_lstm": False,
    "max_seq_len": 20,
    "lstm_cell_size": 256,
    "lstm_use_prev_action": False,
    "lstm_use_prev_reward": False,
    "use_attention": False,
    "framestack": True,
    "dim": 84,
    "grayscale": False,
    "zero_mean": True,
    "custom_model": None,
    "custom_model_config": {},
    "custom_action_dist": None,
    "custom_preprocessor": None,
}


# ----------------------------------------------------------------------------- action distributions
class ActionDistribution:
    def __init__(self, inputs, model=None):
        self.inputs = inputs
        self.model = model

    def sample(self):
        raise NotImplementedError

    def deterministic_sample(self):
        raise NotImplementedError

    def sampled_action_logp(self):
        return self.logp(self._last_sample)

    def logp(self, x):
        raise NotImplementedError

    def kl(self, other):
        raise NotImplementedError

    def entropy(self):
        raise NotImplementedError

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        raise NotImplementedError


class TorchCategorical(ActionDistribution):
    def __init__(self, inputs, model=None):
        super().__init__(inputs, model)
        self._d = Categorical(inputs)

    def sample(self):
        self._last_sample = self._d.sample()
        return self._last_sample

    def deterministic_sample(self):
        self._last_sample = self._d.deterministic_sample()
        return self._last_sample

    def logp(self, x):
        return self._d.logp(x)

    def kl(self, other):
        return self._d.kl(other._d)

    def entropy(self):
        return self._d.entropy()

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        return action_space.n


class TorchDiagGaussian(TorchCategorical):
    def __init__(self, inputs, model=None):
        ActionDistribution.__init__(self, inputs, model)
        self._d = DiagGaussian(inputs)

    @staticmethod
    def required_model_output_shape(action_space, model_config):
        return 2 * int(np.prod(action_space.shape))


# ----------------------------------------------------------------------------- models
class ModelV2:
    """Old-stack model interface: ``forward(input_dict, state, seq_lens) -> (outputs, state)``,
    ``value_function()`` after a forward pass."""

    def __init__(self, obs_space, action_space, num_outputs, model_config, name, framework="torch"):
        self.obs_space, self.action_space = obs_space, action_space
        self.num_outputs = num_outputs
        self.model_config = model_config
        self.name = name
        self.framework = framework
        self.time_major = model_config.get("_time_major", False)

    def get_initial_state(self) -> List:
        return []

    def forward(self, input_dict, state, seq_lens):
        raise NotImplementedError

    def value_function(self):
        raise NotImplementedError

    def custom_loss(self, policy_loss, loss_inputs):
        return policy_loss

    def metrics(self) -> Dict:
        return {}

    def is_time_major(self) -> bool:
        return self.time_major

    def __call__(self, input_dict, state=None, seq_lens=None):
        if not isinstance(input_dict, dict):
            input_dict = {"obs": input_dict}
        input_dict.setdefault("obs_flat", input_dict["obs"].reshape(input_dict["obs"].shape[0], -1)
                              if hasattr(input_dict["obs"], "reshape") else input_dict["obs"])
        return self.forward(input_dict, state or [], seq_lens)


class TorchModelV2(ModelV2):
    """Mix with ``nn.Module``: ``class M(TorchModelV2, nn.Module)`` and call both __init__s."""

    def variables(self, as_dict: bool = False):
        params = dict(self.named_parameters()) if isinstance(self, nn.Module) else {}
        return params if as_dict else list(params.values())

    def trainable_variables(self, as_dict: bool = False):
        v = self.variables(as_dict=True)
        v = {k: p for k, p in v.items() if p.requires_grad}
        return v if as_dict else list(v.values())


class FullyConnectedNetwork(TorchModelV2, nn.Module):
    """The built-in MLP policy / value model (``fcnet_hiddens``, ``fcnet_activation``,
    ``vf_share_layers``)."""

    def __init__(self, obs_space, action_space, num_outputs, model_config, name="fcnet"):
        nn.Module.__init__(self)
        cfg = dict(MODEL_DEFAULTS, **(model_config or {}))
        TorchModelV2.__init__(self, obs_space, action_space, num_outputs, cfg, name)
        inp = int(np.prod(obs_space.shape))
        self._body, feat = _mlp(inp, cfg["fcnet_hiddens"], cfg["fcnet_activation"])
        self._logits = nn.Linear(feat, num_outputs)
        self._vf_body = None if cfg["vf_share_layers"] else _mlp(inp, cfg["fcnet_hiddens"], cfg["fcnet_activation"])[0]
        self._vf = nn.Linear(feat, 1)
        self._features = None
        self._vf_in = None

    def forward(self, input_dict, state, seq_lens):
        x = torch.as_tensor(input_dict["obs_flat"] if "obs_flat" in input_dict else input_dict["obs"]).float()
        x = x.reshape(x.shape[0], -1)
        self._features = self._body(x)
        self._vf_in = x
        return self._logits(self._features), state

    def value_function(self):
        h = self._features if self._vf_body is None else self._vf_body(self._vf_in)
        return self._vf(h).squeeze(-1)


# ----------------------------------------------------------------------------- preprocessors
class Preprocessor:
    def __init__(self, obs_space, options: Optional[Dict] = None):
        self._obs_space = obs_space
        self._options = options or {}
        self.shape = self._init_shape(obs_space, self._options)
        self._size = int(np.prod(self.shape))

    def _init_shape(self, obs_space, options):
        raise NotImplementedError

    def transform(self, observation) -> np.ndarray:
        raise NotImplementedError

    def write(self, observation, array, offset: int) -> None:
        array[offset:offset + self._size] = self.transform(observation).reshape(-1)

    @property
    def size(self) -> int:
        return self._size

    @property
    def observation_space(self):
        return Box(-np.inf, np.inf, self.shape, np.float32)


class NoPreprocessor(Preprocessor):
    def _init_shape(self, obs_space, options):
        return tuple(obs_space.shape)

    def transform(self, observation):
        return np.asarray(observation)


class OneHotPreprocessor(Preprocessor):
    def _init_shape(self, obs_space, options):
        return (obs_space.n,)

    def transform(self, observation):
        out = np.zeros(self.shape, np.float32)
        out[int(observation)] = 1.0
        return out


class FlattenPreprocessor(Preprocessor):
    """Tuple / Dict spaces: each component preprocessed and concatenated."""

    def _init_shape(self, obs_space, options):
        subs = obs_space.spaces if isinstance(obs_space, TupleSpace) else list(obs_space.spaces.values())
        self._subs = [get_preprocessor(s)(s, options) for s in subs]
        return (sum(p.size for p in self._subs),)

    def transform(self, observation):
        parts = observation if isinstance(self._obs_space, TupleSpace) else \
            [observation[k] for k in self._obs_space.spaces]
        return np.concatenate([np.asarray(p.transform(o), np.float32).reshape(-1)
                               for p, o in zip(self._subs, parts)])


def get_preprocessor(space) -> type:
    if isinstance(space, Discrete):
        return OneHotPreprocessor
    if isinstance(space, (TupleSpace, DictSpace)):
        return FlattenPreprocessor
    return NoPreprocessor


# ----------------------------------------------------------------------------- catalog
class ModelCatalog:
    _custom_models: Dict[str, type] = {}
    _custom_action_dists: Dict[str, type] = {}

    @staticmethod
    def register_custom_model(model_name: str, model_class: type) -> None:
        ModelCatalog._custom_models[model_name] = model_class

    @staticmethod
    def register_custom_action_dist(action_dist_name: str, action_dist_class: type) -> None:
        ModelCatalog._custom_action_dists[action_dist_name] = action_dist_class

    @staticmethod
    def get_action_dist(action_space, config: Optional[Dict] = None, dist_type=None, framework: str = "torch",
                        **kw) -> Tuple[type, int]:
        cfg = dict(MODEL_DEFAULTS, **(config or {}))
        if framework != "torch":
            raise ImportError(f"framework={framework!r} is not installed here")
        name = cfg.get("custom_action_dist")
        if name:
            cls = ModelCatalog._custom_action_dists[name]
            return cls, cls.required_model_output_shape(action_space, cfg)
        cls = dist_type or (TorchCategorical if isinstance(action_space, Discrete) else TorchDiagGaussian)
        return cls, cls.required_model_output_shape(action_space, cfg)

    @staticmethod
    def get_model_v2(obs_space, action_space, num_outputs: int, model_config: Dict, framework: str = "torch",
                     name: str = "default_model", model_interface=None, default_model=None, **model_kwargs):
        if framework != "torch":
            raise ImportError(f"framework={framework!r} is not installed here")
        cfg = dict(MODEL_DEFAULTS, **copy.deepcopy(model_config or {}))
        custom = cfg.get("custom_model")
        if custom:
            cls = ModelCatalog._custom_models[custom] if isinstance(custom, str) else custom
            return cls(obs_space, action_space, num_outputs, cfg, name, **cfg.get("custom_model_config", {}),
                       **model_kwargs)
        cls = default_model or FullyConnectedNetwork
        return cls(obs_space, action_space, num_outputs, cfg, name)

    @staticmethod
    def get_preprocessor(env, options: Optional[Dict] = None):
        return ModelCatalog.get_preprocessor_for_space(env.observation_space, options)

    @staticmethod
    def get_preprocessor_for_space(observation_space, options: Optional[Dict] = None) -> Preprocessor:
        opts = dict(MODEL_DEFAULTS, **(options or {}))
        return get_preprocessor(observation_space)(observation_space, opts)


__all__ = ["ActionDistribution", "ModelCatalog", "ModelV2", "Preprocessor", "MODEL_DEFAULTS", "TorchModelV2",
           "FullyConnectedNetwork", "TorchCategorical", "TorchDiagGaussian", "NoPreprocessor",
           "OneHotPreprocessor", "FlattenPreprocessor", "get_preprocessor"]
