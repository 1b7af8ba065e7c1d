"""EpisodeReplayBuffer (reference: ``rllib/utils/replay_buffers/episode_replay_buffer.py:14``).

Stores ``SingleAgentEpisode`` chunks; a chunk whose episode is already in the buffer is appended
to it (``concat_episode``), so an episode sampled across several ``sample()`` rounds is one
trajectory here. Capacity is in env timesteps; whole episodes are evicted oldest first.

Two sampling forms:

* transitions (``batch_length_T=None``, DQN / SAC): ``batch_size_B`` uniformly drawn timesteps
  ``t`` with n-step returns ``sum_k gamma^k r_{t+k}`` over up to ``n_step`` steps (clipped at the
  episode's end), ``new_obs`` = the observation after them and ``n_step`` = how many were
  summed (the learner bootstraps with ``gamma ** n_step``); with ``frame_stack > 1`` both
  observations are the stacks of the last ``frame_stack`` frames read from the episode (zeros
  before its start) -- frame stacking on the learner side from episode data, no stacked frames
  stored;
* sequences (``batch_length_T = T``, DreamerV3-style): ``[B, T]`` windows of consecutive steps
  with ``is_first`` flags.
"""
from __future__ import annotations

import collections
from typing import Dict, List, Optional

import numpy as np

from ...env.single_agent_episode import SingleAgentEpisode
from ...policy.sample_batch import SampleBatch


class EpisodeReplayBuffer:
    def __init__(self, capacity: int = 10000, *, batch_size_B: int = 16, batch_length_T: Optional[int] = None,
                 seed: Optional[int] = None):
        self.capacity = int(capacity)
        self.batch_size_B = int(batch_size_B)
        self.batch_length_T = batch_length_T
        self.episodes: "collections.deque[SingleAgentEpisode]" = collections.deque()
        self.episode_id_to_index: Dict[str, int] = {}
        self._num_timesteps = 0
        self._num_timesteps_added = 0
        self._num_episodes_evicted = 0
        self._offset = 0  # index of episodes[0] in the ever-growing episode numbering
        self._cum = None  # cumulative lengths for uniform timestep sampling (rebuilt lazily)
        self.rng = np.random.default_rng(seed)

    # ------------------------------------------------------------------ adding
    def add(self, episodes):
        if isinstance(episodes, SingleAgentEpisode):
            episodes = [episodes]
        for ep in episodes:
            ep = ep if ep.is_finalized else ep.finalize()
            n = len(ep)
            if n == 0:
                continue
            self._num_timesteps += n
            self._num_timesteps_added += n
            idx = self.episode_id_to_index.get(ep.id_)
            if idx is not None and idx >= self._offset:
                self.episodes[idx - self._offset].concat_episode(ep)
            else:
                self.episode_id_to_index[ep.id_] = self._offset + len(self.episodes)
                self.episodes.append(ep.slice(slice(0, None)) if ep._lb else ep)
        while self._num_timesteps > self.capacity and len(self.episodes) > 1:
            old = self.episodes.popleft()
            self._num_timesteps -= len(old)
            self.episode_id_to_index.pop(old.id_, None)
            self._offset += 1
            self._num_episodes_evicted += 1
        self._cum = None

    # ------------------------------------------------------------------ sampling
    def _index(self):
        if self._cum is None:
            self._cum = np.cumsum([len(e) for e in self.episodes])
        return self._cum

    def get_sampled_timesteps(self) -> int:
        """Timesteps handed out by ``sample`` so far."""
        return getattr(self, "_num_timesteps_sampled", 0)

    def _draw(self, k: int):
        self._num_timesteps_sampled = getattr(self, "_num_timesteps_sampled", 0) + int(k)
        cum = self._index()
        total = int(cum[-1])
        g = self.rng.integers(0, total, k)
        ei = np.searchsorted(cum, g, side="right")
        ts = g - np.concatenate([[0], cum[:-1]])[ei]
        return ei, ts

    def sample(self, num_items: Optional[int] = None, *, batch_size_B: Optional[int] = None,
               batch_length_T: Optional[int] = None, n_step: int = 1, gamma: float = 0.99, frame_stack: int = 1,
               include_extra_model_outputs: bool = False) -> SampleBatch:
        B = int(batch_size_B or num_items or self.batch_size_B)
        T = batch_length_T if batch_length_T is not None else self.batch_length_T
        if not self.episodes:
            raise ValueError("sample() on an empty EpisodeReplayBuffer")
        if T:
            return self._sample_sequences(B, int(T))
        ei, ts = self._draw(B)
        obs, nobs, acts, rews, terms, nst = [], [], [], [], [], []
        extra = collections.defaultdict(list)
        for e_i, t in zip(ei, ts):
            ep = self.episodes[int(e_i)]
            t = int(t)
            n = min(int(n_step), len(ep) - t)
            r = ep.get_rewards(slice(t, t + n))
            ret = float(np.sum(r * gamma ** np.arange(n)))
            if frame_stack > 1:
                obs.append(ep.get_frame_stack(frame_stack, t))
                nobs.append(ep.get_frame_stack(frame_stack, t + n))
            else:
                obs.append(ep.get_observations(t))
                nobs.append(ep.get_observations(t + n))
            acts.append(ep.get_actions(t))
            rews.append(ret)
            terms.append(ep.is_terminated and t + n == len(ep))
            nst.append(n)
            if include_extra_model_outputs:
                for k in ep.extra_model_outputs:
                    extra[k].append(ep.get_extra_model_outputs(k, t))
        b = SampleBatch({SampleBatch.OBS: np.stack(obs), SampleBatch.NEXT_OBS: np.stack(nobs),
                         SampleBatch.ACTIONS: np.stack(acts), SampleBatch.REWARDS: np.asarray(rews, np.float32),
                         SampleBatch.TERMINATEDS: np.asarray(terms, bool),
                         "n_step": np.asarray(nst, np.int64)})
        for k, v in extra.items():
            b[k] = np.stack(v)
        return b

    def _sample_sequences(self, B: int, T: int) -> SampleBatch:
        obs, acts, rews, first, terms = [], [], [], [], []
        for _ in range(B):
            o, a, r, f, d = [], [], [], [], []
            e_i, t = (int(x[0]) for x in self._draw(1))
            while len(a) < T:
                ep = self.episodes[e_i]
                if t == 0 or not a:
                    f.append(t == 0)
                else:
                    f.append(False)
                o.append(ep.get_observations(t))
                a.append(ep.get_actions(t))
                r.append(ep.get_rewards(t))
                d.append(ep.is_terminated and t == len(ep) - 1)
                t += 1
                if t >= len(ep):  # continue in the next (or a random) episode, flagged as a start
                    e_i = int(self.rng.integers(0, len(self.episodes)))
                    t = 0
            obs.append(np.stack(o))
            acts.append(np.stack(a))
            rews.append(np.asarray(r, np.float32))
            first.append(np.asarray(f, bool))
            terms.append(np.asarray(d, bool))
        return SampleBatch({SampleBatch.OBS: np.stack(obs), SampleBatch.ACTIONS: np.stack(acts),
                            SampleBatch.REWARDS: np.stack(rews), "is_first": np.stack(first),
                            SampleBatch.TERMINATEDS: np.stack(terms)})

    # ------------------------------------------------------------------ stats / state
    def __len__(self) -> int:
        return self._num_timesteps

    def get_num_episodes(self) -> int:
        return len(self.episodes)

    def get_num_timesteps(self) -> int:
        return self._num_timesteps

    def get_added_timesteps(self) -> int:
        return self._num_timesteps_added

    def get_state(self) -> Dict:
        return {"episodes": [e.get_state() for e in self.episodes], "offset": self._offset,
                "num_added": self._num_timesteps_added, "evicted": self._num_episodes_evicted}

    def set_state(self, state: Dict):
        self.episodes = collections.deque(SingleAgentEpisode.from_state(s) for s in state["episodes"])
        self._offset = state["offset"]
        self.episode_id_to_index = {e.id_: self._offset + i for i, e in enumerate(self.episodes)}
        self._num_timesteps = sum(len(e) for e in self.episodes)
        self._num_timesteps_added = state["num_added"]
        self._num_episodes_evicted = state["evicted"]
        self._cum = None
