"""DeepMind-style Atari preprocessing wrappers (reference: ``rllib/env/wrappers/atari_wrappers.py``,
the DQN-paper conventions from OpenAI baselines).

They wrap any single env with the gymnasium API that exposes the ALE hooks the conventions need
(``env.unwrapped.ale.lives()``, ``env.unwrapped.get_action_meanings()``, ``env.unwrapped.np_random``).
ALE itself is not installed in this image, so they are exercised on an ALE-shaped test env;
the framework's own vectorised stand-in (``SyntheticAtari-v0``) already renders 84x84x4 stacks.

  * ``NoopResetEnv``: 1..noop_max NOOP steps after every reset (varied start states);
  * ``FireResetEnv``: press FIRE (and action 2) after reset, for games frozen until fired;
  * ``EpisodicLifeEnv``: a lost life ends the episode; the real reset only after game over;
  * ``MaxAndSkipEnv``: repeat the action ``skip`` frames, sum rewards, max-pool the last two frames;
  * ``WarpFrame``: grayscale + area-resize to ``dim x dim x 1`` uint8 (numpy; no OpenCV);
  * ``FrameStack`` / ``FrameStackTrajectoryView``, ``ClipRewardEnv``, ``NormalizedImageEnv``,
    ``MonitorEnv`` (per-episode returns / lengths before life-splitting);
  * ``wrap_deepmind`` / ``wrap_atari_for_new_api_stack``: the standard stacks.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, Optional, Tuple

import numpy as np

from ...utils.spaces import Box
from ..envs import ObservationWrapper, RewardWrapper, Wrapper


def is_atari(env) -> bool:
    """An ``"ALE/..."`` id, or an env object whose repr names an ALE AtariEnv and whose
    observations are images (rank > 2)."""
    if isinstance(env, str):
        return env.startswith("ALE/")
    shape = getattr(getattr(env, "observation_space", None), "shape", None)
    if shape is not None and len(shape) <= 2:
        return False
    return "AtariEnv<ALE" in str(env)


def get_wrapper_by_cls(env, cls):
    """The first wrapper of type ``cls`` going inwards from ``env`` (None if there is none)."""
    cur = env
    while cur is not None:
        if isinstance(cur, cls):
            return cur
        cur = cur.env if isinstance(cur, Wrapper) else None
    return None


def _meanings(env):
    return list(env.unwrapped.get_action_meanings())


def _rng(env):
    r = getattr(env.unwrapped, "np_random", None)
    return r if r is not None else np.random.default_rng()


class ClipRewardEnv(RewardWrapper):
    def reward(self, reward):
        return float(np.sign(reward))


class NoopResetEnv(Wrapper):
    def __init__(self, env, noop_max: int = 30):
        super().__init__(env)
        if _meanings(env)[0] != "NOOP":
            raise ValueError("NoopResetEnv: action 0 must be NOOP")
        self.noop_max = int(noop_max)
        self.noop_action = 0
        self.override_num_noops: Optional[int] = None

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        n = self.override_num_noops
        if n is None:
            r = _rng(self.env)
            n = int(r.integers(1, self.noop_max + 1)) if hasattr(r, "integers") else int(r.randint(1, self.noop_max + 1))
        for _ in range(max(1, n)):
            obs, _, te, tr, info = self.env.step(self.noop_action)
            if te or tr:
                obs, info = self.env.reset(**kwargs)
        return obs, info


class FireResetEnv(Wrapper):
    def __init__(self, env):
        super().__init__(env)
        m = _meanings(env)
        if len(m) < 3 or m[1] != "FIRE":
            raise ValueError("FireResetEnv: action 1 must be FIRE (and the game needs >= 3 actions)")

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        for a in (1, 2):  # FIRE, then one more action some games need to start moving
            obs, _, te, tr, info = self.env.step(a)
            if te or tr:
                obs, info = self.env.reset(**kwargs)
        return obs, info


class EpisodicLifeEnv(Wrapper):
    def __init__(self, env):
        super().__init__(env)
        self.lives = 0
        self.was_real_terminated = True

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        self.was_real_terminated = bool(te)
        lives = self.env.unwrapped.ale.lives()
        if 0 < lives < self.lives:  # a life was lost (lives == 0 is the real game over)
            te = True
        self.lives = lives
        return obs, r, te, tr, info

    def reset(self, **kwargs):
        if self.was_real_terminated:
            obs, info = self.env.reset(**kwargs)
        else:  # continue the same game from the state after the lost life
            obs, _, _, _, info = self.env.step(0)
        self.lives = self.env.unwrapped.ale.lives()
        return obs, info


class MaxAndSkipEnv(Wrapper):
    def __init__(self, env, skip: int = 4):
        super().__init__(env)
        self._skip = int(skip)
        sp = env.observation_space
        self._last2 = np.zeros((2,) + tuple(sp.shape), dtype=sp.dtype)

    def step(self, action):
        total, te, tr, info = 0.0, False, False, {}
        for i in range(self._skip):
            obs, r, te, tr, info = self.env.step(action)
            slot = i - (self._skip - 2)
            if slot >= 0:
                self._last2[slot] = obs
            total += r
            if te or tr:
                break
        return self._last2.max(axis=0), total, te, tr, info


def _area_matrix(n_in: int, n_out: int) -> np.ndarray:
    """[n_out, n_in] weights of area-averaging resampling (each output pixel averages the input
    interval it covers, fractional overlaps weighted)."""
    edges = np.linspace(0.0, n_in, n_out + 1)
    m = np.zeros((n_out, n_in), dtype=np.float32)
    for o in range(n_out):
        a, b = edges[o], edges[o + 1]
        i0, i1 = int(np.floor(a)), int(np.ceil(b))
        for i in range(i0, min(i1, n_in)):
            m[o, i] = min(b, i + 1) - max(a, i)
        m[o] /= m[o].sum()
    return m


class WarpFrame(ObservationWrapper):
    """RGB (or single-channel) frame -> ``dim x dim x 1`` uint8 luminance."""

    _LUMA = np.array([0.299, 0.587, 0.114], dtype=np.float32)

    def __init__(self, env, dim: int = 84):
        super().__init__(env)
        self.width = self.height = int(dim)
        self.observation_space = Box(0, 255, shape=(self.height, self.width, 1), dtype=np.uint8)
        self._mats: Dict[Tuple[int, int], Tuple[np.ndarray, np.ndarray]] = {}

    def observation(self, frame):
        f = np.asarray(frame, dtype=np.float32)
        gray = f @ self._LUMA if f.ndim == 3 and f.shape[-1] == 3 else f.reshape(f.shape[0], f.shape[1])
        key = gray.shape
        if key not in self._mats:
            self._mats[key] = (_area_matrix(key[0], self.height), _area_matrix(key[1], self.width).T)
        mh, mw = self._mats[key]
        out = mh @ gray @ mw
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)[:, :, None]


class NormalizedImageEnv(ObservationWrapper):
    """uint8 frames -> float32 in [-1, 1)."""

    def __init__(self, env):
        super().__init__(env)
        self.observation_space = Box(-1.0, 1.0, shape=env.observation_space.shape, dtype=np.float32)

    def observation(self, observation):
        return np.asarray(observation, dtype=np.float32) / 128.0 - 1.0


class FrameStack(Wrapper):
    """The last ``k`` frames concatenated on the channel axis (the first frame repeated after reset)."""

    def __init__(self, env, k: int):
        super().__init__(env)
        self.k = int(k)
        self.frames: deque = deque(maxlen=self.k)
        sp = env.observation_space
        h, w, c = sp.shape
        self.observation_space = Box(np.repeat(sp.low, self.k, axis=-1), np.repeat(sp.high, self.k, axis=-1),
                                     shape=(h, w, c * self.k), dtype=sp.dtype)

    def reset(self, **kwargs):
        ob, info = self.env.reset(**kwargs)
        self.frames.extend([ob] * self.k)
        return self._stack(), info

    def step(self, action):
        ob, r, te, tr, info = self.env.step(action)
        self.frames.append(ob)
        return self._stack(), r, te, tr, info

    def _stack(self):
        return np.concatenate(list(self.frames), axis=-1)


class FrameStackTrajectoryView(ObservationWrapper):
    """``h x w x 1`` -> ``h x w`` (the connector / view requirements stack frames instead)."""

    def __init__(self, env):
        super().__init__(env)
        h, w, c = env.observation_space.shape
        if c != 1:
            raise ValueError("FrameStackTrajectoryView expects single-channel frames")
        self.observation_space = Box(0, 255, shape=(h, w), dtype=env.observation_space.dtype)

    def observation(self, observation):
        return np.squeeze(observation, axis=-1)


class MonitorEnv(Wrapper):
    """Episode returns / lengths of the underlying game, recorded before any life-splitting."""

    def __init__(self, env=None):
        super().__init__(env)
        self._ret: Optional[float] = None
        self._len = 0
        self._total: Optional[int] = None
        self._returns: list = []
        self._lengths: list = []
        self._num_returned = 0

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        if self._total is None:
            self._total = sum(self._lengths)
        if self._ret is not None:
            self._returns.append(self._ret)
            self._lengths.append(self._len)
        self._ret, self._len = 0.0, 0
        return obs, info

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        self._ret += r
        self._len += 1
        self._total += 1
        return obs, r, te, tr, info

    def get_episode_rewards(self):
        return self._returns

    def get_episode_lengths(self):
        return self._lengths

    def get_total_steps(self):
        return self._total

    def next_episode_results(self):
        new = list(zip(self._returns[self._num_returned:], self._lengths[self._num_returned:]))
        self._num_returned = len(self._returns)
        yield from new


def wrap_deepmind(env, dim: int = 84, framestack: bool = True, noframeskip: bool = False):
    """The DQN-paper stack: monitor, no-op starts, (frame skip for NoFrameskip games), life
    episodes, fire-on-reset, 84x84 grayscale, 4-frame stack. Reward clipping is left to the
    algorithm (e.g. the ClipRewards connector)."""
    env = MonitorEnv(env)
    env = NoopResetEnv(env, noop_max=30)
    if getattr(env, "spec", None) is not None and noframeskip is True:
        env = MaxAndSkipEnv(env, skip=4)
    env = EpisodicLifeEnv(env)
    if "FIRE" in _meanings(env):
        env = FireResetEnv(env)
    env = WarpFrame(env, dim)
    if framestack is True:
        env = FrameStack(env, 4)
    return env


class _TimeLimit(Wrapper):
    def __init__(self, env, max_episode_steps: int):
        super().__init__(env)
        self._max, self._t = int(max_episode_steps), 0

    def reset(self, **kwargs):
        self._t = 0
        return self.env.reset(**kwargs)

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        self._t += 1
        return obs, r, te, tr or self._t >= self._max, info


def wrap_atari_for_new_api_stack(env, dim: int = 64, frameskip: int = 4, framestack: Optional[int] = None):
    """The new-API-stack Atari stack: 108k-step time limit, ``dim x dim`` grayscale normalised to
    [-1, 1], frame skip with max-pooling, no-op starts, life episodes, fire-on-reset and an
    optional frame stack (after the skip)."""
    env = _TimeLimit(env, max_episode_steps=108000)
    env = WarpFrame(env, dim=dim)
    env = NormalizedImageEnv(env)
    if frameskip > 1:
        env = MaxAndSkipEnv(env, skip=frameskip)
    env = NoopResetEnv(env, noop_max=30)
    env = EpisodicLifeEnv(env)
    if "FIRE" in _meanings(env):
        env = FireResetEnv(env)
    if framestack:
        env = FrameStack(env, k=framestack)
    return env


__all__ = ["is_atari", "get_wrapper_by_cls", "ClipRewardEnv", "NoopResetEnv", "FireResetEnv", "EpisodicLifeEnv",
           "MaxAndSkipEnv", "WarpFrame", "NormalizedImageEnv", "FrameStack", "FrameStackTrajectoryView",
           "MonitorEnv", "wrap_deepmind", "wrap_atari_for_new_api_stack"]
