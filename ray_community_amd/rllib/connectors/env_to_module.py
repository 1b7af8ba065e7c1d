"""Env -> module connector pieces (reference: ``rllib/connectors/env_to_module/``:
``flatten_observations.py``, ``mean_std_filter.py``, ``prev_actions_prev_rewards.py``,
``frame_stacking.py``). Each operates on ``batch["obs"]`` = numpy ``[N, ...]`` of the N
vectorised sub-envs; per-env history rows reset where ``episodes.is_first`` is set."""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np

from ..utils.spaces import Box, Discrete
from .connector_v2 import ConnectorV2


def _flat_dim(space) -> int:
    return int(np.prod(space.shape)) if space is not None and space.shape else 1


class FlattenObservations(ConnectorV2):
    """``[N, *shape]`` -> ``[N, prod(shape)]`` float32."""

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None:
            return None
        lo = np.asarray(obs_space.low, dtype=np.float32).reshape(-1)
        hi = np.asarray(obs_space.high, dtype=np.float32).reshape(-1)
        return Box(lo, hi, dtype=np.float32)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        o = np.asarray(batch["obs"])
        batch["obs"] = o.reshape(o.shape[0], -1).astype(np.float32, copy=False)
        return batch


class MeanStdFilter(ConnectorV2):
    """Running mean / std normalisation of observations, optionally clipped.

    Statistics are a synced ``base`` (Welford count / mean / M2) plus this runner's ``delta``
    since the last sync; ``merge_states`` combines the bases with every runner's delta (parallel
    Welford) so no sample is counted twice, and ``set_state`` installs the merged base and clears
    the delta."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, clip_by_value: float = 10.0,
                 de_mean_observations: bool = True, de_std_observations: bool = True, update_stats: bool = True,
                 epsilon: float = 1e-8, **kw):
        self.clip = clip_by_value
        self.de_mean, self.de_std = de_mean_observations, de_std_observations
        self.update_stats = update_stats
        self.eps = epsilon
        self.base = None
        self.delta = None
        super().__init__(input_observation_space, input_action_space, **kw)

    @staticmethod
    def _empty(shape):
        return {"n": 0.0, "mean": np.zeros(shape, np.float64), "m2": np.zeros(shape, np.float64)}

    @staticmethod
    def _combine(a, b):
        n = a["n"] + b["n"]
        if n == 0:
            return {"n": 0.0, "mean": a["mean"].copy(), "m2": a["m2"].copy()}
        d = b["mean"] - a["mean"]
        mean = a["mean"] + d * (b["n"] / n)
        m2 = a["m2"] + b["m2"] + d * d * (a["n"] * b["n"] / n)
        return {"n": n, "mean": mean, "m2": m2}

    def _ensure(self, shape):
        if self.base is None or self.base["mean"].shape != shape:
            self.base, self.delta = self._empty(shape), self._empty(shape)

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None:
            return None
        c = self.clip if self.clip else np.inf
        return Box(-c, c, shape=obs_space.shape, dtype=np.float32)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        o = np.asarray(batch["obs"], dtype=np.float64)
        self._ensure(o.shape[1:])
        if self.update_stats and not (shared_data or {}).get("peek"):
            x = {"n": float(o.shape[0]), "mean": o.mean(0), "m2": ((o - o.mean(0)) ** 2).sum(0)}
            self.delta = self._combine(self.delta, x)
        st = self._combine(self.base, self.delta)
        y = o
        if self.de_mean:
            y = y - st["mean"]
        if self.de_std and st["n"] > 1:
            y = y / (np.sqrt(st["m2"] / st["n"]) + self.eps)
        if self.clip:
            y = np.clip(y, -self.clip, self.clip)
        batch["obs"] = y.astype(np.float32)
        return batch

    def get_state(self, components=None, *, not_components=None, **kw):
        return {"base": self.base, "delta": self.delta}

    def set_state(self, state):
        if state and state.get("base") is not None:
            self.base = {k: (np.array(v) if k != "n" else float(v)) for k, v in state["base"].items()}
            self.delta = self._empty(self.base["mean"].shape)

    def reset_state(self):
        self.base = self.delta = None

    @classmethod
    def merge_states(cls, states: List[Dict[str, Any]]) -> Dict[str, Any]:
        states = [s for s in states if s and s.get("base") is not None]
        if not states:
            return {"base": None, "delta": None}
        merged = dict(states[0]["base"])
        for s in states:
            merged = cls._combine(merged, s["delta"])
        return {"base": merged, "delta": cls._empty(merged["mean"].shape)}

    @property
    def running_mean(self):
        return None if self.base is None else self._combine(self.base, self.delta)["mean"]


class PrevActionsPrevRewards(ConnectorV2):
    """Appends the last ``n_prev_actions`` actions (one-hot for Discrete) and ``n_prev_rewards``
    rewards of each sub-env to its (flattened) observation; zeros at episode start."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, n_prev_actions: int = 1,
                 n_prev_rewards: int = 1, **kw):
        self.na, self.nr = int(n_prev_actions), int(n_prev_rewards)
        self.ha = None  # [N, na, A]
        self.hr = None  # [N, nr]
        super().__init__(input_observation_space, input_action_space, **kw)

    def _adim(self):
        s = self._input_action_space
        return s.n if isinstance(s, Discrete) else _flat_dim(s)

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None or act_space is None:
            return obs_space
        d = _flat_dim(obs_space) + self.na * (act_space.n if isinstance(act_space, Discrete) else _flat_dim(act_space))
        d += self.nr
        return Box(-np.inf, np.inf, shape=(d,), dtype=np.float32)

    def _encode(self, a):
        s = self._input_action_space
        a = np.asarray(a)
        if isinstance(s, Discrete):
            out = np.zeros((a.shape[0], s.n), np.float32)
            out[np.arange(a.shape[0]), a.astype(np.int64).reshape(-1)] = 1.0
            return out
        return a.reshape(a.shape[0], -1).astype(np.float32)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        o = np.asarray(batch["obs"], dtype=np.float32)
        n = o.shape[0]
        peek = bool((shared_data or {}).get("peek"))
        A = self._adim()
        if self.ha is None:
            N = episodes.num_envs if episodes is not None and episodes.env_indices is None else n
            self.ha = np.zeros((N, self.na, A), np.float32)
            self.hr = np.zeros((N, self.nr), np.float32)
        idx = episodes.env_indices if episodes is not None and episodes.env_indices is not None else slice(None)
        ha, hr = self.ha[idx].copy(), self.hr[idx].copy()
        if episodes is not None and episodes.last_actions is not None:
            if self.na:
                ha = np.concatenate([ha[:, 1:], self._encode(episodes.last_actions)[:, None]], axis=1)
            if self.nr:
                hr = np.concatenate([hr[:, 1:], np.asarray(episodes.last_rewards, np.float32)[:, None]], axis=1)
        if episodes is not None:
            first = np.asarray(episodes.is_first, dtype=bool)
            ha[first] = 0.0
            hr[first] = 0.0
        if not peek:
            self.ha[idx], self.hr[idx] = ha, hr
        batch["obs"] = np.concatenate([o.reshape(n, -1), ha.reshape(n, -1), hr], axis=1)
        return batch

    def reset_state(self):
        self.ha = self.hr = None


class FrameStackingEnvToModule(ConnectorV2):
    """Stacks each sub-env's last ``num_frames`` observations along the last axis (the first
    observation of an episode fills every slot)."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, num_frames: int = 4, **kw):
        self.k = int(num_frames)
        self.hist = None  # [N, k, *obs_shape]
        super().__init__(input_observation_space, input_action_space, **kw)

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None:
            return None
        lo = np.concatenate([np.asarray(obs_space.low)] * self.k, axis=-1)
        hi = np.concatenate([np.asarray(obs_space.high)] * self.k, axis=-1)
        return Box(lo, hi, dtype=obs_space.dtype)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None, **kw):
        o = np.asarray(batch["obs"])
        peek = bool((shared_data or {}).get("peek"))
        idx = episodes.env_indices if episodes is not None and episodes.env_indices is not None else slice(None)
        if self.hist is None:
            self.hist = np.repeat(o[:, None], self.k, axis=1)
            h = self.hist.copy()
        else:
            h = np.concatenate([self.hist[idx][:, 1:], o[:, None]], axis=1)
            if episodes is not None:
                first = np.asarray(episodes.is_first, dtype=bool)
                if first.any():
                    h[first] = np.repeat(o[first][:, None], self.k, axis=1)
            if not peek:
                self.hist[idx] = h
        batch["obs"] = np.concatenate([h[:, i] for i in range(self.k)], axis=-1)
        return batch

    def reset_state(self):
        self.hist = None

# the reference package's default pieces (see connectors/common.py)
from .common import (AddObservationsFromEpisodesToBatch, AddStatesFromEpisodesToBatch, AgentToModuleMapping, BatchIndividualItems, NumpyToTensor, WriteObservationsToEpisodes)  # noqa: E402,F401
from .connector_v2 import EnvToModulePipeline  # noqa: E402,F401

PrevActionsPrevRewardsConnector = PrevActionsPrevRewards
