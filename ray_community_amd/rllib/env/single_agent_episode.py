"""SingleAgentEpisode: one agent's trajectory chunk (reference: ``rllib/env/single_agent_episode.py:18``).

The episode holds observations (one more than actions: the reset observation starts it), actions,
rewards, infos and extra model outputs (e.g. ``action_logp``, ``vf_preds``) of the env steps
``t_started .. t``. A chunk may carry a LOOKBACK buffer: the last ``len_lookback_buffer`` steps of
the previous chunk of the same episode, readable through negative indices with
``neg_index_as_lookback=True`` -- what frame stacking and n-step returns read across a chunk
boundary. Index semantics of ``get_*`` (``indices`` = int, list or slice):

* non-negative indices count from the first step of THIS chunk (0 = its first observation);
* negative indices count from the end (-1 = the latest item) unless ``neg_index_as_lookback``,
  in which case -1 is the last item BEFORE the chunk (the lookback buffer's newest entry);
* ``fill``: indices outside the data return ``fill`` instead of raising (zero-padding at an
  episode's start, e.g. the first frames of a stack).

``finalize()`` converts the lists to numpy arrays (the form replay buffers keep); ``cut()`` starts
the next chunk with a lookback; ``concat_episode()`` appends a continuation chunk;
``to_sample_batch()`` gives the classic transition batch (obs, new_obs, ...).
"""
from __future__ import annotations

import uuid
from typing import Any, Dict, List, Optional

import numpy as np


class SingleAgentEpisode:
    def __init__(self, id_: Optional[str] = None, *, observations: Optional[List] = None,
                 actions: Optional[List] = None, rewards: Optional[List] = None, infos: Optional[List] = None,
                 terminated: bool = False, truncated: bool = False,
                 extra_model_outputs: Optional[Dict[str, List]] = None, t_started: int = 0,
                 len_lookback_buffer: int = 0, observation_space=None, action_space=None, agent_id=None,
                 module_id=None, multi_agent_episode_id: Optional[str] = None):
        self.id_ = id_ or uuid.uuid4().hex
        self.agent_id = agent_id
        self.module_id = module_id
        self.multi_agent_episode_id = multi_agent_episode_id
        self.observation_space = observation_space
        self.action_space = action_space
        self.observations = list(observations) if observations is not None else []
        self.actions = list(actions) if actions is not None else []
        self.rewards = list(rewards) if rewards is not None else []
        self.infos = list(infos) if infos is not None else [{} for _ in self.observations]
        self.extra_model_outputs = {k: list(v) for k, v in (extra_model_outputs or {}).items()}
        self.is_terminated = bool(terminated)
        self.is_truncated = bool(truncated)
        # lookback: the first ``_lb`` actions/rewards (and observations) precede t_started
        self._lb = int(len_lookback_buffer)
        self.t_started = int(t_started)
        self.t = self.t_started + max(0, len(self.actions) - self._lb)
        self.is_finalized = False
        self._custom = {}

    # ------------------------------------------------------------------ building
    def add_env_reset(self, observation, infos: Optional[Dict] = None):
        if self.observations:
            raise ValueError("add_env_reset on an episode that already has observations")
        self.observations.append(observation)
        self.infos.append(dict(infos or {}))

    def add_env_step(self, observation, action, reward: float, infos: Optional[Dict] = None, *,
                     terminated: bool = False, truncated: bool = False,
                     extra_model_outputs: Optional[Dict[str, Any]] = None):
        if self.is_done:
            raise ValueError(f"episode {self.id_} is done: no more steps")
        if self.is_finalized:
            raise ValueError("add_env_step on a finalized episode")
        self.observations.append(observation)
        self.actions.append(action)
        self.rewards.append(float(reward))
        self.infos.append(dict(infos or {}))
        for k, v in (extra_model_outputs or {}).items():
            self.extra_model_outputs.setdefault(k, [None] * (len(self.actions) - 1)).append(v)
        self.t += 1
        self.is_terminated = bool(terminated)
        self.is_truncated = bool(truncated)

    def finalize(self) -> "SingleAgentEpisode":
        """Lists -> numpy arrays (observations / actions / rewards / extra model outputs)."""
        if self.is_finalized:
            return self
        self.observations = _stack(self.observations)
        self.actions = _stack(self.actions)
        self.rewards = np.asarray(self.rewards, dtype=np.float32)
        self.extra_model_outputs = {k: _stack(v) for k, v in self.extra_model_outputs.items()}
        self.is_finalized = True
        return self

    def validate(self):
        n = len(self.actions)
        if len(self.observations) != n + 1 and not (n == 0 and len(self.observations) <= 1):
            raise AssertionError(f"{len(self.observations)} observations for {n} actions")
        if len(self.rewards) != n:
            raise AssertionError(f"{len(self.rewards)} rewards for {n} actions")
        for k, v in self.extra_model_outputs.items():
            if len(v) != n:
                raise AssertionError(f"extra model output {k!r}: {len(v)} entries for {n} actions")

    # ------------------------------------------------------------------ properties
    @property
    def is_done(self) -> bool:
        return self.is_terminated or self.is_truncated

    @property
    def is_reset(self) -> bool:
        return len(self.observations) > 0

    def __len__(self) -> int:
        return self.t - self.t_started

    def env_steps(self) -> int:
        return len(self)

    def agent_steps(self) -> int:
        return len(self)

    def get_return(self, include_hanging_rewards: bool = False) -> float:
        return float(np.sum(np.asarray(self.rewards, dtype=np.float64)[self._lb:]))

    def get_duration_s(self) -> float:
        return float(self._custom.get("_duration_s", 0.0))

    # ------------------------------------------------------------------ access
    def _resolve(self, n_items: int, lb: int, indices, neg_index_as_lookback: bool, fill):
        """Absolute positions (into the stored list of ``n_items`` with ``lb`` lookback items) of
        ``indices``; out-of-range -> None (filled) or IndexError."""
        single = indices is not None and not isinstance(indices, (list, tuple, slice, range, np.ndarray))
        if indices is None:
            idx = list(range(lb, n_items))
        elif isinstance(indices, slice):
            start, stop, step = indices.start, indices.stop, indices.step or 1
            if neg_index_as_lookback:
                rng = range(lb + (start if start is not None else 0),
                            lb + (stop if stop is not None else n_items - lb), step)
            else:
                norm = lambda i, d: d if i is None else (i + n_items if i < 0 else lb + i)  # noqa: E731
                rng = range(norm(start, lb), norm(stop, n_items), step)
            idx = list(rng)
        else:
            seq = [indices] if single else list(indices)
            idx = []
            for i in seq:
                i = int(i)
                if i >= 0:
                    idx.append(lb + i)
                elif neg_index_as_lookback:
                    idx.append(lb + i)
                else:
                    idx.append(n_items + i)
        out = []
        for a in idx:
            if 0 <= a < n_items:
                out.append(a)
            elif fill is not None:
                out.append(None)
            else:
                raise IndexError(f"index out of range of episode {self.id_} (length {n_items - lb}, lookback {lb})")
        return out, single

    def _get(self, data, lb, indices, neg_index_as_lookback, fill):
        n = len(data)
        pos, single = self._resolve(n, lb, indices, neg_index_as_lookback, fill)
        items = []
        for a in pos:
            if a is None:
                ref = data[0] if n else None
                items.append(_fill_like(ref, fill))
            else:
                items.append(data[a])
        if single:
            return items[0]
        return _stack(items) if self.is_finalized or (items and isinstance(items[0], np.ndarray)) else items

    def get_observations(self, indices=None, *, neg_index_as_lookback: bool = False, fill=None):
        return self._get(self.observations, self._lb, indices, neg_index_as_lookback, fill)

    def get_actions(self, indices=None, *, neg_index_as_lookback: bool = False, fill=None):
        return self._get(self.actions, self._lb, indices, neg_index_as_lookback, fill)

    def get_rewards(self, indices=None, *, neg_index_as_lookback: bool = False, fill=None):
        r = self._get(self.rewards, self._lb, indices, neg_index_as_lookback, fill)
        return np.asarray(r, dtype=np.float32) if not np.isscalar(r) else r

    def get_infos(self, indices=None, *, neg_index_as_lookback: bool = False, fill=None):
        return self._get(self.infos, self._lb, indices, neg_index_as_lookback, fill)

    def get_extra_model_outputs(self, key: str, indices=None, *, neg_index_as_lookback: bool = False, fill=None):
        return self._get(self.extra_model_outputs[key], self._lb, indices, neg_index_as_lookback, fill)

    def get_frame_stack(self, num_frames: int, index: int = -1) -> np.ndarray:
        """The ``num_frames`` observations ending at ``index`` (chunk-relative, -1 = latest),
        concatenated on the last axis; frames before the episode's start are zeros."""
        n = len(self.observations)
        end = (n + index) if index < 0 else self._lb + index
        frames = [self.observations[a] if a >= 0 else None for a in range(end - num_frames + 1, end + 1)]
        ref = next(f for f in frames if f is not None)
        frames = [np.zeros_like(np.asarray(ref)) if f is None else np.asarray(f) for f in frames]
        return np.concatenate(frames, axis=-1)

    # ------------------------------------------------------------------ chunks
    def cut(self, len_lookback_buffer: int = 0) -> "SingleAgentEpisode":
        """The continuation chunk: starts at this chunk's last observation (t), carrying the last
        ``len_lookback_buffer`` steps as lookback."""
        if self.is_done:
            raise ValueError("cut() on a done episode")
        k = min(int(len_lookback_buffer), len(self.actions))
        obs = list(self.observations[len(self.observations) - 1 - k:])
        acts = list(self.actions[len(self.actions) - k:]) if k else []
        rews = list(self.rewards[len(self.rewards) - k:]) if k else []
        infos = list(self.infos[len(self.infos) - 1 - k:])
        extra = {key: (list(v[len(v) - k:]) if k else []) for key, v in self.extra_model_outputs.items()}
        return SingleAgentEpisode(self.id_, observations=obs, actions=acts, rewards=rews, infos=infos,
                                  extra_model_outputs=extra, t_started=self.t, len_lookback_buffer=k,
                                  observation_space=self.observation_space, action_space=self.action_space,
                                  agent_id=self.agent_id, module_id=self.module_id,
                                  multi_agent_episode_id=self.multi_agent_episode_id)

    def concat_episode(self, other: "SingleAgentEpisode"):
        """Append the continuation chunk ``other`` (same id, starting where this one ends)."""
        if other.id_ != self.id_:
            raise ValueError("concat_episode needs a chunk of the same episode")
        if other.t_started != self.t:
            raise ValueError(f"chunk starts at t={other.t_started}, this one ends at t={self.t}")
        if self.is_done:
            raise ValueError("concat_episode onto a done episode")
        was = self.is_finalized
        if was:
            self._unfinalize()
        olb = other._lb
        o_obs = list(other.observations)[olb + 1:]
        self.observations = list(self.observations) + o_obs
        self.actions = list(self.actions) + list(other.actions)[olb:]
        self.rewards = list(self.rewards) + list(other.rewards)[olb:]
        self.infos = list(self.infos) + list(other.infos)[olb + 1:]
        for k, v in other.extra_model_outputs.items():
            self.extra_model_outputs[k] = list(self.extra_model_outputs.get(k, [])) + list(v)[olb:]
        self.t = other.t
        self.is_terminated, self.is_truncated = other.is_terminated, other.is_truncated
        if was:
            self.finalize()

    def _unfinalize(self):
        self.observations = list(self.observations)
        self.actions = list(self.actions)
        self.rewards = list(self.rewards)
        self.extra_model_outputs = {k: list(v) for k, v in self.extra_model_outputs.items()}
        self.is_finalized = False

    def slice(self, slice_: slice, *, len_lookback_buffer: int = 0) -> "SingleAgentEpisode":
        """Steps ``slice_`` (chunk-relative, step 1) as a new chunk of the same episode."""
        start = 0 if slice_.start is None else (slice_.start if slice_.start >= 0 else len(self) + slice_.start)
        stop = len(self) if slice_.stop is None else (slice_.stop if slice_.stop >= 0 else len(self) + slice_.stop)
        start, stop = max(0, start), min(len(self), stop)
        k = min(len_lookback_buffer, start + self._lb)
        a0 = self._lb + start
        obs = list(self.observations[a0 - k: self._lb + stop + 1])
        acts = list(self.actions[a0 - k: self._lb + stop])
        rews = list(self.rewards[a0 - k: self._lb + stop])
        infos = list(self.infos[a0 - k: self._lb + stop + 1])
        extra = {key: list(v[a0 - k: self._lb + stop]) for key, v in self.extra_model_outputs.items()}
        done_here = stop == len(self)
        ep = SingleAgentEpisode(self.id_, observations=obs, actions=acts, rewards=rews, infos=infos,
                                extra_model_outputs=extra, t_started=self.t_started + start, len_lookback_buffer=k,
                                terminated=self.is_terminated and done_here,
                                truncated=self.is_truncated and done_here,
                                observation_space=self.observation_space, action_space=self.action_space,
                                agent_id=self.agent_id, module_id=self.module_id,
                                multi_agent_episode_id=self.multi_agent_episode_id)
        if self.is_finalized:
            ep.finalize()
        return ep

    # ------------------------------------------------------------------ in-place edits
    def _set(self, data, new_data, at_indices, neg_index_as_lookback):
        pos, single = self._resolve(len(data), self._lb, at_indices, neg_index_as_lookback, None)
        vals = [new_data] if single else list(new_data)
        if len(vals) != len(pos):
            raise IndexError(f"{len(vals)} new items for {len(pos)} positions")
        for a, v in zip(pos, vals):
            data[a] = v

    def set_observations(self, *, new_data, at_indices=None, neg_index_as_lookback: bool = False):
        """Overwrite stored observations (same index rules as ``get_observations``)."""
        self._set(self.observations, new_data, at_indices, neg_index_as_lookback)

    def set_actions(self, *, new_data, at_indices=None, neg_index_as_lookback: bool = False):
        self._set(self.actions, new_data, at_indices, neg_index_as_lookback)

    def set_rewards(self, *, new_data, at_indices=None, neg_index_as_lookback: bool = False):
        self._set(self.rewards, new_data, at_indices, neg_index_as_lookback)

    def set_extra_model_outputs(self, *, key, new_data, at_indices=None, neg_index_as_lookback: bool = False):
        self._set(self.extra_model_outputs[key], new_data, at_indices, neg_index_as_lookback)

    # ------------------------------------------------------------------ conversion
    def get_data_dict(self) -> Dict[str, Any]:
        """The episode's columns (no lookback), one row per timestep (``SampleBatch`` keys)."""
        return {k: v for k, v in self.to_sample_batch().items()}

    def get_sample_batch(self):
        return self.to_sample_batch()

    def to_sample_batch(self):
        from ..policy.sample_batch import SampleBatch

        n = len(self)
        lb = self._lb
        obs = _stack(list(self.observations)[lb: lb + n + 1])
        d = {SampleBatch.OBS: obs[:n], SampleBatch.NEXT_OBS: obs[1: n + 1],
             SampleBatch.ACTIONS: _stack(list(self.actions)[lb:]),
             SampleBatch.REWARDS: np.asarray(list(self.rewards)[lb:], dtype=np.float32),
             SampleBatch.TERMINATEDS: np.zeros(n, dtype=bool), SampleBatch.TRUNCATEDS: np.zeros(n, dtype=bool),
             SampleBatch.EPS_ID: np.full(n, hash(self.id_) & 0x7FFFFFFF, dtype=np.int64),
             SampleBatch.T: np.arange(self.t_started, self.t, dtype=np.int64)}
        if n:
            d[SampleBatch.TERMINATEDS][-1] = self.is_terminated
            d[SampleBatch.TRUNCATEDS][-1] = self.is_truncated
        for k, v in self.extra_model_outputs.items():
            d[k] = _stack(list(v)[lb:])
        return SampleBatch(d)

    def get_state(self) -> Dict[str, Any]:
        return {"id_": self.id_, "agent_id": self.agent_id, "module_id": self.module_id,
                "multi_agent_episode_id": self.multi_agent_episode_id,
                "observations": list(self.observations), "actions": list(self.actions),
                "rewards": list(self.rewards), "infos": list(self.infos),
                "extra_model_outputs": {k: list(v) for k, v in self.extra_model_outputs.items()},
                "terminated": self.is_terminated, "truncated": self.is_truncated, "t_started": self.t_started,
                "t": self.t, "len_lookback_buffer": self._lb, "is_finalized": self.is_finalized}

    @staticmethod
    def from_state(state: Dict[str, Any]) -> "SingleAgentEpisode":
        ep = SingleAgentEpisode(state["id_"], observations=state["observations"], actions=state["actions"],
                                rewards=state["rewards"], infos=state["infos"],
                                extra_model_outputs=state["extra_model_outputs"], terminated=state["terminated"],
                                truncated=state["truncated"], t_started=state["t_started"],
                                len_lookback_buffer=state["len_lookback_buffer"], agent_id=state["agent_id"],
                                module_id=state["module_id"],
                                multi_agent_episode_id=state["multi_agent_episode_id"])
        if state.get("is_finalized"):
            ep.finalize()
        return ep

    def __repr__(self):
        return (f"SAEps(len={len(self)} done={self.is_done} R={self.get_return():.2f} id_={self.id_[:8]} "
                f"t={self.t_started}..{self.t})")


def _stack(items):
    if isinstance(items, np.ndarray):
        return items
    if not len(items):
        return np.zeros((0,), dtype=np.float32)
    try:
        return np.stack([np.asarray(x) for x in items])
    except ValueError:
        arr = np.empty(len(items), dtype=object)
        arr[:] = items
        return arr


def _fill_like(ref, fill):
    if ref is None:
        return fill
    r = np.asarray(ref)
    if r.shape == ():
        return type(ref)(fill) if isinstance(ref, (int, float)) else fill
    return np.full_like(r, fill)
