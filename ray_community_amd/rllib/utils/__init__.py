"""RLlib utilities (reference: rllib/utils/__init__.py and the modules it re-exports:
annotations, framework, numpy, schedules, filter, test_utils, deprecation).

Framework probes: only torch is installed here, so ``try_import_tf`` / ``try_import_tfp`` /
``try_import_jax`` return ``None`` placeholders the way the reference does when a framework is
missing, and ``framework_iterator`` yields "torch" only."""
from __future__ import annotations

import copy
import warnings
from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np

from .filter import Filter, FilterManager, MeanStdFilter, NoFilter
from .schedules import (ConstantSchedule, ExponentialSchedule, LinearSchedule, PiecewiseSchedule,
                        PolynomialSchedule)

LARGE_INTEGER = 100000000
SMALL_NUMBER = 1e-6
MIN_LOG_NN_OUTPUT = -5
MAX_LOG_NN_OUTPUT = 2


# ------------------------------------------------------------------------- annotations
def override(parent_cls):
    """Marks a method as overriding one of ``parent_cls`` (checked at decoration time)."""
    def deco(method):
        if not hasattr(parent_cls, method.__name__):
            raise NameError(f"{method.__name__} does not override any method of {parent_cls.__name__}")
        return method
    return deco


def PublicAPI(obj=None, **kw):  # noqa: N802 (reference name)
    return obj if obj is not None else (lambda o: o)


DeveloperAPI = PublicAPI


def deprecation_warning(old: str, new: Optional[str] = None, *, help: Optional[str] = None,
                        error: bool = False) -> None:
    msg = f"`{old}` has been deprecated." + (f" Use `{new}` instead." if new else "") + (f" {help}" if help else "")
    if error:
        raise ValueError(msg)
    warnings.warn(msg, DeprecationWarning, stacklevel=2)


# ------------------------------------------------------------------------- framework probes
def try_import_torch(error: bool = False):
    import torch
    import torch.nn as nn

    return torch, nn


def try_import_tf(error: bool = False):
    if error:
        raise ImportError("TensorFlow is not installed in this environment")
    return None, None, None


def try_import_tfp(error: bool = False):
    if error:
        raise ImportError("tensorflow_probability is not installed in this environment")
    return None


def try_import_jax(error: bool = False):
    if error:
        raise ImportError("JAX is not installed in this environment")
    return None, None


def framework_iterator(config=None, frameworks: Sequence[str] = ("torch",), session: bool = False, **kw):
    """Yields each requested framework that is installed (torch only here), setting
    ``config["framework"]`` / ``config.framework_str`` as it goes."""
    for fw in frameworks:
        if fw != "torch":
            continue
        if config is not None:
            if isinstance(config, dict):
                config["framework"] = fw
            elif hasattr(config, "framework"):
                config.framework(fw)
        yield fw


# ------------------------------------------------------------------------- dict / list helpers
def deep_update(original: Dict, new_dict: Dict, new_keys_allowed: bool = True,
                allow_new_subkey_list: Optional[List[str]] = None,
                override_all_if_type_changes: Optional[List[str]] = None,
                override_all_key_list: Optional[List[str]] = None) -> Dict:
    """Recursively update ``original`` in place with ``new_dict`` (returns it)."""
    allow_new_subkey_list = allow_new_subkey_list or []
    override_all_if_type_changes = override_all_if_type_changes or []
    override_all_key_list = override_all_key_list or []
    for k, value in new_dict.items():
        if k not in original and not new_keys_allowed:
            raise Exception(f"Unknown config parameter `{k}` ")
        if isinstance(original.get(k), dict) and isinstance(value, dict):
            if k in override_all_key_list:
                original[k] = value
            elif k in override_all_if_type_changes and "type" in value and "type" in original[k] \
                    and value["type"] != original[k]["type"]:
                original[k] = value
            else:
                deep_update(original[k], value, k in allow_new_subkey_list or new_keys_allowed,
                            allow_new_subkey_list, override_all_if_type_changes, override_all_key_list)
        else:
            original[k] = value
    return original


def merge_dicts(d1: Dict, d2: Dict) -> Dict:
    """A deep copy of ``d1`` updated recursively with ``d2``."""
    return deep_update(copy.deepcopy(d1), d2, True)


def force_list(elements=None, to_tuple: bool = False):
    ctor = tuple if to_tuple else list
    if elements is None:
        return ctor()
    if isinstance(elements, (list, tuple, set)):
        return ctor(elements)
    return ctor([elements])


def force_tuple(elements=None):
    return force_list(elements, to_tuple=True)


def add_mixins(base, mixins: Iterable, reversed: bool = False):  # noqa: A002 (reference name)
    """A subclass of ``base`` with ``mixins`` mixed in (first mixin has the highest priority)."""
    mixins = list(mixins or [])
    if reversed:
        mixins = mixins[::-1]
    if not mixins:
        return base
    return type(base.__name__, tuple(mixins) + (base,), {})


# ------------------------------------------------------------------------- numpy math
def one_hot(x, depth: int = 0, on_value: float = 1.0, off_value: float = 0.0, dtype=np.float32):
    x = np.asarray(x)
    depth = int(depth or (int(x.max()) + 1 if x.size else 1))
    out = np.full(x.shape + (depth,), off_value, dtype=dtype)
    np.put_along_axis(out, x[..., None].astype(np.int64), on_value, axis=-1)
    return out


def softmax(x, axis: int = -1, epsilon: Optional[float] = None):
    x = np.asarray(x, dtype=np.float64)
    e = np.exp(x - x.max(axis=axis, keepdims=True))
    out = e / e.sum(axis=axis, keepdims=True)
    return np.maximum(out, epsilon) if epsilon else out


def sigmoid(x, derivative: bool = False):
    s = 1.0 / (1.0 + np.exp(-np.asarray(x, dtype=np.float64)))
    return s * (1 - s) if derivative else s


def relu(x, alpha: float = 0.0):
    x = np.asarray(x)
    return np.maximum(x, x * alpha)


def fc(x, weights, biases=None, framework: Optional[str] = None):
    """Dense layer in numpy: ``x @ W + b`` (torch tensors are converted)."""
    def _np(v):
        return v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
    out = _np(x) @ _np(weights)
    return out + _np(biases) if biases is not None else out


def lstm(x, weights, biases=None, initial_internal_states=None, time_major: bool = False,
         forget_bias: float = 1.0):
    """A numpy LSTM over ``x`` [B, T, in] (or [T, B, in] if time_major) with fused gate weights
    [in + units, 4 units] in (i, j(candidate), f, o) order; returns (outputs, (c, h))."""
    x = np.asarray(x, dtype=np.float64)
    if time_major:
        x = x.transpose(1, 0, 2)
    B, T, _ = x.shape
    units = weights.shape[1] // 4
    c, h = (np.zeros((B, units)), np.zeros((B, units))) if initial_internal_states is None else \
        (np.asarray(initial_internal_states[0], np.float64), np.asarray(initial_internal_states[1], np.float64))
    b = np.zeros(4 * units) if biases is None else np.asarray(biases)
    outs = np.zeros((B, T, units))
    for t in range(T):
        z = np.concatenate([x[:, t], h], axis=1) @ weights + b
        i, j, f, o = np.split(z, 4, axis=1)
        c = c * sigmoid(f + forget_bias) + sigmoid(i) * np.tanh(j)
        h = np.tanh(c) * sigmoid(o)
        outs[:, t] = h
    if time_major:
        outs = outs.transpose(1, 0, 2)
    return outs, (c, h)


# ------------------------------------------------------------------------- test utils
def check(x, y, decimals: int = 5, atol: Optional[float] = None, rtol: Optional[float] = None,
          false: bool = False) -> None:
    """Nested-structure equality with numeric tolerance (``false=True`` asserts inequality)."""
    def _cmp(a, b):
        if isinstance(a, dict):
            assert isinstance(b, dict) and set(a) == set(b), f"dict keys differ: {set(a) ^ set(b)}"
            for k in a:
                _cmp(a[k], b[k])
            return
        if isinstance(a, (list, tuple)) and not np.isscalar(a):
            assert len(a) == len(b), f"lengths differ: {len(a)} vs {len(b)}"
            for u, v in zip(a, b):
                _cmp(u, v)
            return
        if hasattr(a, "detach"):
            a = a.detach().cpu().numpy()
        if hasattr(b, "detach"):
            b = b.detach().cpu().numpy()
        a, b = np.asarray(a), np.asarray(b)
        if a.dtype.kind in "fc" or b.dtype.kind in "fc":
            if atol is None and rtol is None:
                np.testing.assert_almost_equal(a, b, decimal=decimals)
            else:
                np.testing.assert_allclose(a, b, atol=atol or 0, rtol=rtol or 1e-7)
        else:
            np.testing.assert_array_equal(a, b)
    if false:
        try:
            _cmp(x, y)
        except AssertionError:
            return
        raise AssertionError(f"{x} and {y} are equal, expected them to differ")
    _cmp(x, y)


def check_train_results(train_results: Dict) -> Dict:
    """Basic shape checks of an ``Algorithm.train()`` result dict."""
    for key in ("training_iteration", "timesteps_total") if "timesteps_total" in train_results else \
            ("training_iteration",):
        assert key in train_results, f"'{key}' missing from train results"
    return train_results


def check_compute_single_action(algorithm, include_state: bool = False, include_prev_action_reward: bool = False):
    """``compute_single_action`` on a sampled observation returns an action of the action space."""
    runner = getattr(algorithm, "local_runner", None) or getattr(algorithm, "env_runner", None)
    space = None
    if runner is not None and hasattr(runner, "spaces"):
        obs_space, space = runner.spaces()
        obs = obs_space.sample()
    else:
        obs = np.zeros(4, np.float32)
    a = algorithm.compute_single_action(obs)
    if space is not None and hasattr(space, "contains"):
        assert space.contains(a), f"action {a!r} not in {space}"
    return a


def check_env(env, config: Optional[Dict] = None) -> None:
    """Sanity checks of a (gym-style or multi-agent) env: reset / step return shapes and spaces."""
    from ..env.multi_agent_env import MultiAgentEnv

    if isinstance(env, MultiAgentEnv):
        obs, infos = env.reset()
        assert isinstance(obs, dict), "MultiAgentEnv.reset must return a dict of observations"
        acts = {aid: env.get_action_space(aid).sample() if hasattr(env, "get_action_space")
                else env.action_space.sample() for aid in obs}
        out = env.step(acts)
        assert len(out) == 5 and all(isinstance(o, dict) for o in out), "step must return 5 dicts"
        assert "__all__" in out[2], "terminateds must have an '__all__' key"
        return
    reset = env.reset()
    obs = reset[0] if isinstance(reset, tuple) else reset
    space = getattr(env, "observation_space", None)
    if space is not None and hasattr(space, "contains"):
        assert space.contains(np.asarray(obs)[0] if np.ndim(obs) > len(space.shape) else obs), \
            "reset observation not in observation_space"
    a = env.action_space.sample()
    out = env.step(a)
    assert len(out) == 5, "step must return (obs, reward, terminated, truncated, info)"


__all__ = ["override", "PublicAPI", "DeveloperAPI", "deprecation_warning", "try_import_torch", "try_import_tf",
           "try_import_tfp", "try_import_jax", "framework_iterator", "deep_update", "merge_dicts", "force_list",
           "force_tuple", "add_mixins", "one_hot", "softmax", "sigmoid", "relu", "fc", "lstm", "check",
           "check_train_results", "check_compute_single_action", "check_env", "Filter", "FilterManager",
           "MeanStdFilter", "NoFilter", "ConstantSchedule", "ExponentialSchedule", "LinearSchedule",
           "PiecewiseSchedule", "PolynomialSchedule", "LARGE_INTEGER", "SMALL_NUMBER", "MIN_LOG_NN_OUTPUT",
           "MAX_LOG_NN_OUTPUT"]
