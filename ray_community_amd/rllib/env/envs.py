"""Environments: a gymnasium-style single-env API plus natively vectorised numpy envs.

gymnasium / ALE are not installed in this environment, so the framework ships:
  * ``CartPole-v1`` and ``Pendulum-v1`` (classic-control dynamics, vectorised over N envs);
  * ``StatelessCartPole-v1`` (CartPole without the velocities: needs a memory-based policy);
  * ``SyntheticAtari-v0`` — an Atari-shaped task (84x84x4 uint8 frame stacks, Discrete(6)
    actions, +/-1 rewards): a falling-ball "catch" game rendered into 84x84 frames, used as the
    shape-faithful stand-in for ALE games (``ALE/*`` ids resolve to it, flagged in ``info``).
Custom envs: ``register_env(name, creator)`` with a gym-like object exposing
``reset() -> (obs, info)`` and ``step(a) -> (obs, r, terminated, truncated, info)``.
Reference: ``rllib/env/{vector_env,single_agent_env_runner}.py`` and gymnasium semantics.
"""
from __future__ import annotations

import math
import os
import sys
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np

from ..utils.spaces import Box, Discrete

_REGISTRY: Dict[str, Callable] = {}


def register_env(name: str, creator: Callable):
    _REGISTRY[name] = creator


class Env:
    observation_space = None
    action_space = None
    metadata = {}

    def reset(self, *, seed=None, options=None):
        raise NotImplementedError

    def step(self, action):
        raise NotImplementedError

    def close(self):
        pass

    @property
    def unwrapped(self):
        return self


class Wrapper(Env):
    """gymnasium-style wrapper: delegates to ``self.env``; spaces default to the wrapped env's and
    unknown attributes are looked up on it (``wrapper.unwrapped`` is the innermost env)."""

    def __init__(self, env):
        self.env = env
        self.observation_space = getattr(env, "observation_space", None)
        self.action_space = getattr(env, "action_space", None)

    def __getattr__(self, name):
        if name.startswith("_") or name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return getattr(self.env, "unwrapped", self.env)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        return self.env.step(action)

    def close(self):
        close = getattr(self.env, "close", None)
        if close is not None:
            close()


class ObservationWrapper(Wrapper):
    def observation(self, observation):
        raise NotImplementedError

    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        return self.observation(obs), info

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        return self.observation(obs), r, te, tr, info


class RewardWrapper(Wrapper):
    def reward(self, reward):
        raise NotImplementedError

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        return obs, self.reward(r), te, tr, info


class VectorEnv:
    """N environments stepped as one batch. ``step`` auto-resets finished sub-envs and returns the
    pre-reset observation in ``info["final_obs"]`` (row-aligned, valid where done)."""

    num_envs: int
    observation_space = None
    action_space = None

    def reset(self, seed=None):
        raise NotImplementedError

    def step(self, actions):
        raise NotImplementedError


class CartPoleVec(VectorEnv):
    def __init__(self, num_envs=1, max_episode_steps=500, seed=None):
        self.num_envs = num_envs
        self.gravity, self.masscart, self.masspole, self.length = 9.8, 1.0, 0.1, 0.5
        self.total_mass = self.masscart + self.masspole
        self.polemass_length = self.masspole * self.length
        self.force_mag, self.tau = 10.0, 0.02
        self.theta_th = 12 * 2 * math.pi / 360
        self.x_th = 2.4
        high = np.array([self.x_th * 2, np.finfo(np.float32).max, self.theta_th * 2, np.finfo(np.float32).max],
                        dtype=np.float32)
        self.observation_space = Box(-high, high, dtype=np.float32)
        self.action_space = Discrete(2)
        self.max_steps = max_episode_steps
        self.rng = np.random.default_rng(seed)
        self.state = np.zeros((num_envs, 4), dtype=np.float64)
        self.t = np.zeros(num_envs, dtype=np.int64)

    def _render_packed(self, idx, all_envs):
        pk = self._packed
        by = np.clip(self.by[idx].astype(np.int64), 0, self.H - 2)
        bx = np.clip(self.bx[idx].astype(np.int64), 0, self.W - 2)
        px = np.clip(self.px[idx].astype(np.int64), 6, self.W - 7)
        if all_envs:
            pk >>= 8  # drop the oldest frame; the new frame's byte starts black
            rows = idx
        else:
            sub = pk[idx]
            sub >>= 8
            pk[idx] = sub
            rows = idx
        top = np.uint32(255 << 24)
        for dy in (0, 1):
            for dx in (0, 1):
                pk[rows, by + dy, bx + dx] |= top
        # the paddle is drawn after the ball and overwrites it where they overlap
        keep, pad = np.uint32(0x00FFFFFF), np.uint32(200 << 24)
        cols = px[:, None] + np.arange(-6, 7)[None, :]
        r2 = np.broadcast_to(rows[:, None], cols.shape)
        for y in (self.H - 2, self.H - 1):
            pk[r2, y, cols] = (pk[r2, y, cols] & keep) | pad

    def reset(self, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.state = self.rng.uniform(-0.05, 0.05, size=(self.num_envs, 4))
        self.t[:] = 0
        return self.state.astype(np.float32), {}

    def step(self, actions):
        a = np.asarray(actions).reshape(-1)
        x, x_dot, th, th_dot = self.state.T
        force = np.where(a == 1, self.force_mag, -self.force_mag)
        ct, st = np.cos(th), np.sin(th)
        temp = (force + self.polemass_length * th_dot ** 2 * st) / self.total_mass
        thacc = (self.gravity * st - ct * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * ct ** 2 / self.total_mass))
        xacc = temp - self.polemass_length * thacc * ct / self.total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        th = th + self.tau * th_dot
        th_dot = th_dot + self.tau * thacc
        self.state = np.stack([x, x_dot, th, th_dot], axis=1)
        self.t += 1
        term = (x < -self.x_th) | (x > self.x_th) | (th < -self.theta_th) | (th > self.theta_th)
        trunc = (self.t >= self.max_steps) & ~term
        rew = np.ones(self.num_envs, dtype=np.float32)
        obs = self.state.astype(np.float32)
        done = term | trunc
        final = obs.copy()
        if done.any():
            n = int(done.sum())
            self.state[done] = self.rng.uniform(-0.05, 0.05, size=(n, 4))
            self.t[done] = 0
            obs = self.state.astype(np.float32)
        return obs, rew, term, trunc, {"final_obs": final}


class StatelessCartPoleVec(CartPoleVec):
    """CartPole with the velocities masked out (observation = [x, theta]): only a policy with
    memory (LSTM, frame stacking or previous-action inputs) can infer the dynamics. Reference:
    ``rllib/examples/envs/classes/stateless_cartpole.py``."""

    def __init__(self, num_envs=1, max_episode_steps=500, seed=None):
        super().__init__(num_envs, max_episode_steps, seed)
        high = np.array([self.x_th * 2, self.theta_th * 2], dtype=np.float32)
        self.observation_space = Box(-high, high, dtype=np.float32)

    def reset(self, seed=None):
        obs, info = super().reset(seed)
        return obs[:, [0, 2]], info

    def step(self, actions):
        obs, rew, term, trunc, info = super().step(actions)
        return obs[:, [0, 2]], rew, term, trunc, {"final_obs": info["final_obs"][:, [0, 2]]}


class PendulumVec(VectorEnv):
    def __init__(self, num_envs=1, max_episode_steps=200, seed=None):
        self.num_envs = num_envs
        self.max_speed, self.max_torque, self.dt, self.g, self.m, self.l = 8.0, 2.0, 0.05, 10.0, 1.0, 1.0
        self.observation_space = Box(np.array([-1, -1, -8.0]), np.array([1, 1, 8.0]), dtype=np.float32)
        self.action_space = Box(-2.0, 2.0, shape=(1,), dtype=np.float32)
        self.max_steps = max_episode_steps
        self.rng = np.random.default_rng(seed)
        self.th = np.zeros(num_envs)
        self.thd = np.zeros(num_envs)
        self.t = np.zeros(num_envs, dtype=np.int64)

    def _obs(self):
        return np.stack([np.cos(self.th), np.sin(self.th), self.thd], axis=1).astype(np.float32)

    def _render_packed(self, idx, all_envs):
        pk = self._packed
        by = np.clip(self.by[idx].astype(np.int64), 0, self.H - 2)
        bx = np.clip(self.bx[idx].astype(np.int64), 0, self.W - 2)
        px = np.clip(self.px[idx].astype(np.int64), 6, self.W - 7)
        if all_envs:
            pk >>= 8  # drop the oldest frame; the new frame's byte starts black
            rows = idx
        else:
            sub = pk[idx]
            sub >>= 8
            pk[idx] = sub
            rows = idx
        top = np.uint32(255 << 24)
        for dy in (0, 1):
            for dx in (0, 1):
                pk[rows, by + dy, bx + dx] |= top
        # the paddle is drawn after the ball and overwrites it where they overlap
        keep, pad = np.uint32(0x00FFFFFF), np.uint32(200 << 24)
        cols = px[:, None] + np.arange(-6, 7)[None, :]
        r2 = np.broadcast_to(rows[:, None], cols.shape)
        for y in (self.H - 2, self.H - 1):
            pk[r2, y, cols] = (pk[r2, y, cols] & keep) | pad

    def reset(self, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.th = self.rng.uniform(-np.pi, np.pi, self.num_envs)
        self.thd = self.rng.uniform(-1, 1, self.num_envs)
        self.t[:] = 0
        return self._obs(), {}

    def step(self, actions):
        u = np.clip(np.asarray(actions, dtype=np.float64).reshape(self.num_envs, -1)[:, 0], -self.max_torque,
                    self.max_torque)
        thn = ((self.th + np.pi) % (2 * np.pi)) - np.pi
        cost = thn ** 2 + 0.1 * self.thd ** 2 + 0.001 * u ** 2
        self.thd = np.clip(self.thd + (3 * self.g / (2 * self.l) * np.sin(self.th) + 3.0 / (self.m * self.l ** 2) * u)
                           * self.dt, -self.max_speed, self.max_speed)
        self.th = self.th + self.thd * self.dt
        self.t += 1
        trunc = self.t >= self.max_steps
        term = np.zeros(self.num_envs, dtype=bool)
        obs = self._obs()
        final = obs.copy()
        if trunc.any():
            n = int(trunc.sum())
            self.th[trunc] = self.rng.uniform(-np.pi, np.pi, n)
            self.thd[trunc] = self.rng.uniform(-1, 1, n)
            self.t[trunc] = 0
            obs = self._obs()
        return obs, (-cost).astype(np.float32), term, trunc, {"final_obs": final}


class SyntheticAtariVec(VectorEnv):
    """Atari-shaped catch game: 84x84 frames, 4-frame stack (HWC uint8), Discrete(6) (NOOP, FIRE,
    RIGHT, LEFT, RIGHTFIRE, LEFTFIRE as in Pong's action set). A ball falls one row per step
    (randomised start column and drift); the paddle on the bottom rows catches it (+1) or misses
    (-1); an episode is ``balls_per_episode`` balls."""

    H = W = 84
    STACK = 4

    def __init__(self, num_envs=1, balls_per_episode=5, max_episode_steps=10000, seed=None, frameskip=1,
                 frame_stack=4):
        """``frame_stack=1``: single frames, for a FrameStacking env-to-module connector to stack
        (the reference's Atari setup); 4 (default): the env stacks them itself."""
        self.num_envs = num_envs
        self.STACK = int(frame_stack)
        self.observation_space = Box(0, 255, shape=(self.H, self.W, self.STACK), dtype=np.uint8)
        self.action_space = Discrete(6)
        self.balls = balls_per_episode
        self.max_steps = max_episode_steps
        self.rng = np.random.default_rng(seed)
        n = num_envs
        self.frames = np.zeros((n, self.H, self.W, self.STACK), dtype=np.uint8)
        # 4-frame stacks as one little-endian uint32 per pixel (byte k = frame k, oldest first):
        # pushing a frame is ONE in-place shift of the packed words plus the new frame's few lit
        # pixels in the top byte, instead of a strided per-channel shift of the HWC uint8 stack
        # (the runner's env step was 30 % of its sample loop, profiles/rllib_runner_r6.md)
        self._packed = self.frames.view(np.uint32).reshape(n, self.H, self.W) \
            if (self.STACK == 4 and sys.byteorder == "little"
                and os.environ.get("RCA_SYNTH_ATARI_PACKED", "1") != "0") else None
        self.bx = np.zeros(n)
        self.by = np.zeros(n)
        self.vx = np.zeros(n)
        self.px = np.full(n, self.W / 2)
        self.left = np.zeros(n, dtype=np.int64)
        self.t = np.zeros(n, dtype=np.int64)
        self._ar = np.arange(n)

    def _new_ball(self, idx):
        k = len(idx) if hasattr(idx, "__len__") else int(np.sum(idx))
        self.bx[idx] = self.rng.uniform(4, self.W - 4, k)
        self.by[idx] = 0.0
        self.vx[idx] = self.rng.uniform(-1.0, 1.0, k)

    def _render(self, mask=None):
        idx = self._ar if mask is None else np.nonzero(mask)[0]
        if len(idx) == 0:
            return
        if self._packed is not None:
            self._render_packed(idx, mask is None)
            return
        f = np.zeros((len(idx), self.H, self.W), dtype=np.uint8)
        by = np.clip(self.by[idx].astype(np.int64), 0, self.H - 2)
        bx = np.clip(self.bx[idx].astype(np.int64), 0, self.W - 2)
        px = np.clip(self.px[idx].astype(np.int64), 6, self.W - 7)
        rr = np.arange(len(idx))
        for dy in (0, 1):
            for dx in (0, 1):
                f[rr, by + dy, bx + dx] = 255
        for dx in range(-6, 7):
            f[rr, self.H - 2, px + dx] = 200
            f[rr, self.H - 1, px + dx] = 200
        fr = self.frames[idx]
        fr[..., :-1] = fr[..., 1:]
        fr[..., -1] = f
        self.frames[idx] = fr

    def _render_packed(self, idx, all_envs):
        pk = self._packed
        by = np.clip(self.by[idx].astype(np.int64), 0, self.H - 2)
        bx = np.clip(self.bx[idx].astype(np.int64), 0, self.W - 2)
        px = np.clip(self.px[idx].astype(np.int64), 6, self.W - 7)
        if all_envs:
            pk >>= 8  # drop the oldest frame; the new frame's byte starts black
            rows = idx
        else:
            sub = pk[idx]
            sub >>= 8
            pk[idx] = sub
            rows = idx
        top = np.uint32(255 << 24)
        for dy in (0, 1):
            for dx in (0, 1):
                pk[rows, by + dy, bx + dx] |= top
        # the paddle is drawn after the ball and overwrites it where they overlap
        keep, pad = np.uint32(0x00FFFFFF), np.uint32(200 << 24)
        cols = px[:, None] + np.arange(-6, 7)[None, :]
        r2 = np.broadcast_to(rows[:, None], cols.shape)
        for y in (self.H - 2, self.H - 1):
            pk[r2, y, cols] = (pk[r2, y, cols] & keep) | pad

    def reset(self, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self._new_ball(self._ar)
        self.px[:] = self.W / 2
        self.left[:] = self.balls
        self.t[:] = 0
        self.frames[:] = 0
        for _ in range(self.STACK):
            self._render()
        return self.frames.copy(), {"synthetic_atari": True}

    def step(self, actions):
        a = np.asarray(actions).reshape(-1)
        move = np.where(np.isin(a, (2, 4)), 3.0, np.where(np.isin(a, (3, 5)), -3.0, 0.0))
        self.px = np.clip(self.px + move, 6, self.W - 7)
        self.bx = np.clip(self.bx + self.vx, 1, self.W - 3)
        self.vx = np.where((self.bx <= 1) | (self.bx >= self.W - 3), -self.vx, self.vx)
        self.by += 2.0
        self.t += 1
        rew = np.zeros(self.num_envs, dtype=np.float32)
        landed = self.by >= self.H - 3
        if landed.any():
            hit = np.abs(self.bx - self.px) <= 7
            rew[landed & hit] = 1.0
            rew[landed & ~hit] = -1.0
            self.left[landed] -= 1
            self._new_ball(landed)
        term = self.left <= 0
        trunc = (self.t >= self.max_steps) & ~term
        self._render()
        obs = self.frames.copy()
        done = term | trunc
        final = obs
        if done.any():
            final = obs.copy()
            self.left[done] = self.balls
            self.t[done] = 0
            self.px[done] = self.W / 2
            self.frames[done] = 0
            for _ in range(self.STACK):
                self._render(done)
            obs = self.frames.copy()
        return obs, rew, term, trunc, {"final_obs": final, "synthetic_atari": True}


class SingleToVector(VectorEnv):
    """Wrap N independent gym-style envs into the VectorEnv interface."""

    def __init__(self, make_env: Callable, num_envs: int, seed=None):
        self.envs = [make_env() for _ in range(num_envs)]
        self.num_envs = num_envs
        self.observation_space = self.envs[0].observation_space
        self.action_space = self.envs[0].action_space
        self._seed = seed

    def reset(self, seed=None):
        obs = []
        for i, e in enumerate(self.envs):
            s = None if seed is None and self._seed is None else (seed or self._seed) + i
            o, _ = e.reset(seed=s)
            obs.append(o)
        return np.stack(obs), {}

    def step(self, actions):
        obs, rew, term, trunc, finals = [], [], [], [], []
        for e, a in zip(self.envs, actions):
            o, r, te, tr, _ = e.step(a)
            finals.append(o)
            if te or tr:
                o, _ = e.reset()
            obs.append(o)
            rew.append(r)
            term.append(te)
            trunc.append(tr)
        return (np.stack(obs), np.asarray(rew, dtype=np.float32), np.asarray(term), np.asarray(trunc),
                {"final_obs": np.stack(finals)})


def make_vector_env(env, num_envs: int, env_config: Optional[dict] = None, seed=None) -> VectorEnv:
    from .env_context import EnvContext

    cfg = env_config if isinstance(env_config, EnvContext) else dict(env_config or {})
    if isinstance(env, str):
        if env in _REGISTRY:
            return SingleToVector(lambda: _REGISTRY[env](cfg), num_envs, seed)
        if env == "CartPole-v1" or env == "CartPole-v0":
            return CartPoleVec(num_envs, max_episode_steps=500 if env.endswith("1") else 200, seed=seed)
        if env in ("StatelessCartPole-v1", "StatelessCartPole"):
            return StatelessCartPoleVec(num_envs, max_episode_steps=int(cfg.get("max_episode_steps", 500)), seed=seed)
        if env == "Pendulum-v1":
            return PendulumVec(num_envs, seed=seed)
        if env.startswith("ALE/") or env == "SyntheticAtari-v0" or "NoFrameskip" in env:
            return SyntheticAtariVec(num_envs, seed=seed, **{k: v for k, v in cfg.items()
                                                             if k in ("balls_per_episode", "max_episode_steps",
                                                                      "frame_stack")})
        raise ValueError(f"unknown env {env!r}; register it with register_env()")
    if isinstance(env, type) and issubclass(env, VectorEnv):
        return env(num_envs=num_envs, **cfg)
    if callable(env):
        return SingleToVector(lambda: env(cfg) if _takes_arg(env) else env(), num_envs, seed)
    raise ValueError(f"unsupported env spec {env!r}")


def _takes_arg(f):
    import inspect

    try:
        return len(inspect.signature(f).parameters) >= 1
    except (TypeError, ValueError):
        return True
