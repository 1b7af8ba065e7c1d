"""Multi-agent environments (reference: ``rllib/env/multi_agent_env.py:29``).

A ``MultiAgentEnv`` speaks dicts keyed by agent id::

    obs, infos = env.reset(seed=...)                       # {agent_id: obs}, {agent_id: info}
    obs, rewards, terminateds, truncateds, infos = env.step({agent_id: action})

``terminateds`` / ``truncateds`` carry per-agent flags plus ``"__all__"`` (the episode is over
for everyone). Agents present in ``obs`` are the ones expected to act next step.
``make_multi_agent`` turns a single-agent env (a registered id or creator) into N independent
agents stepping simultaneously -- the reference's ``make_multi_agent`` helper.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional, Union

import numpy as np


class MultiAgentEnv:
    possible_agents: list = []
    agents: list = []
    observation_spaces: Dict[Any, Any] = {}
    action_spaces: Dict[Any, Any] = {}
    # single spaces shared by every agent (optional alternative to the dicts)
    observation_space = None
    action_space = None

    def reset(self, *, seed=None, options=None):
        raise NotImplementedError

    def step(self, action_dict):
        raise NotImplementedError

    def get_observation_space(self, agent_id):
        return self.observation_spaces.get(agent_id, self.observation_space) if self.observation_spaces \
            else self.observation_space

    def get_action_space(self, agent_id):
        return self.action_spaces.get(agent_id, self.action_space) if self.action_spaces else self.action_space

    def close(self):
        pass

    # reference MultiAgentEnv helpers (rllib/env/multi_agent_env.py)
    def get_agent_ids(self) -> set:
        return set(self.possible_agents or self.agents or self.observation_spaces or ())

    def observation_space_sample(self, agent_ids=None) -> Dict:
        ids = agent_ids if agent_ids is not None else self.get_agent_ids()
        return {a: self.get_observation_space(a).sample() for a in ids}

    def action_space_sample(self, agent_ids=None) -> Dict:
        ids = agent_ids if agent_ids is not None else self.get_agent_ids()
        return {a: self.get_action_space(a).sample() for a in ids}

    def observation_space_contains(self, x: Dict) -> bool:
        return isinstance(x, dict) and all(self.get_observation_space(a).contains(v) for a, v in x.items())

    def action_space_contains(self, x: Dict) -> bool:
        return isinstance(x, dict) and all(self.get_action_space(a).contains(v) for a, v in x.items())

    def render(self):
        return None

    def with_agent_groups(self, groups: Dict, obs_space=None, act_space=None) -> "MultiAgentEnv":
        """Agents grouped into super-agents (reference ``with_agent_groups``): group id -> list of
        agent ids; a group observes / acts with the tuple of its members' observations / actions
        and receives the sum of their rewards."""
        return _GroupedAgents(self, groups, obs_space, act_space)

    def to_base_env(self, make_env=None, num_envs: int = 1, remote_envs: bool = False,
                    remote_env_batch_wait_ms: int = 0, restart_failed_sub_environments: bool = False):
        from .base_env import convert_to_base_env

        return convert_to_base_env(self, make_env=make_env, num_envs=num_envs)


class _GroupedAgents(MultiAgentEnv):
    def __init__(self, env: MultiAgentEnv, groups: Dict, obs_space=None, act_space=None):
        self.env = env
        self.groups = {g: list(m) for g, m in groups.items()}
        grouped = {a for m in self.groups.values() for a in m}
        self._single = [a for a in env.get_agent_ids() if a not in grouped]
        self.possible_agents = list(self.groups) + self._single
        self.agents = list(self.possible_agents)
        self._obs_space, self._act_space = obs_space, act_space

    def get_observation_space(self, agent_id):
        if agent_id in self.groups:
            if self._obs_space is not None:
                return self._obs_space
            from ..utils.spaces import Tuple as _Tuple

            return _Tuple([self.env.get_observation_space(a) for a in self.groups[agent_id]])
        return self.env.get_observation_space(agent_id)

    def get_action_space(self, agent_id):
        if agent_id in self.groups:
            if self._act_space is not None:
                return self._act_space
            from ..utils.spaces import Tuple as _Tuple

            return _Tuple([self.env.get_action_space(a) for a in self.groups[agent_id]])
        return self.env.get_action_space(agent_id)

    def _group_dict(self, d, reduce=None):
        out = {}
        for g, members in self.groups.items():
            vals = [d[a] for a in members if a in d]
            if vals:
                out[g] = reduce(vals) if reduce else tuple(vals)
        for a in self._single:
            if a in d:
                out[a] = d[a]
        return out

    def reset(self, *, seed=None, options=None):
        obs, infos = self.env.reset(seed=seed, options=options)
        return self._group_dict(obs), self._group_dict(infos, reduce=lambda v: v[0])

    def step(self, action_dict):
        flat = {}
        for k, a in action_dict.items():
            if k in self.groups:
                for member, act in zip(self.groups[k], a):
                    flat[member] = act
            else:
                flat[k] = a
        obs, rew, term, trunc, infos = self.env.step(flat)
        o = self._group_dict(obs)
        r = self._group_dict(rew, reduce=lambda v: float(sum(v)))
        te = self._group_dict({k: v for k, v in term.items() if k != "__all__"}, reduce=all)
        tr = self._group_dict({k: v for k, v in trunc.items() if k != "__all__"}, reduce=all)
        te["__all__"] = term.get("__all__", False)
        tr["__all__"] = trunc.get("__all__", False)
        return o, r, te, tr, self._group_dict(infos, reduce=lambda v: v[0])


def make_multi_agent(env_name_or_creator: Union[str, Callable]) -> Callable[[Optional[dict]], MultiAgentEnv]:
    """Class factory: ``make_multi_agent("CartPole-v1")({"num_agents": 2})`` -> an env whose agents
    0..N-1 each run an independent copy of the single-agent env."""

    def build(config: Optional[dict] = None) -> MultiAgentEnv:
        return _IndependentAgents(env_name_or_creator, dict(config or {}))

    return build


class _IndependentAgents(MultiAgentEnv):
    def __init__(self, base, config):
        from .envs import make_vector_env

        n = int(config.pop("num_agents", 2))
        self.possible_agents = [f"agent_{i}" for i in range(n)]
        self._envs = {}
        for i, aid in enumerate(self.possible_agents):
            if callable(base):
                self._envs[aid] = _SingleAsVector(base(config))
            else:
                self._envs[aid] = make_vector_env(base, 1, config)
        first = self._envs[self.possible_agents[0]]
        self.observation_space = first.observation_space
        self.action_space = first.action_space
        self.agents = []
        self._done = {}

    def reset(self, *, seed=None, options=None):
        obs = {}
        for i, (aid, e) in enumerate(self._envs.items()):
            o, _ = e.reset(seed=None if seed is None else seed + 7919 * i)
            obs[aid] = o[0]
        self.agents = list(self.possible_agents)
        self._done = {a: False for a in self.possible_agents}
        return obs, {a: {} for a in obs}

    def step(self, action_dict):
        obs, rew, term, trunc, info = {}, {}, {}, {}, {}
        for aid, a in action_dict.items():
            if self._done.get(aid, True):
                continue
            o, r, te, tr, inf = self._envs[aid].step(np.asarray([a]))
            rew[aid] = float(r[0])
            term[aid] = bool(te[0])
            trunc[aid] = bool(tr[0])
            info[aid] = {}
            if te[0] or tr[0]:
                self._done[aid] = "term" if te[0] else "trunc"
                obs[aid] = inf["final_obs"][0]
            else:
                obs[aid] = o[0]
        self.agents = [a for a in self.possible_agents if not self._done[a]]
        all_done = all(self._done.values())
        term["__all__"] = all_done and any(h == "term" for h in self._done.values())
        trunc["__all__"] = all_done and not term["__all__"]
        return obs, rew, term, trunc, info


class _SingleAsVector:
    """A gym-like single env behind the 1-wide vector interface used by ``_IndependentAgents``."""

    def __init__(self, env):
        self.env = env
        self.observation_space = env.observation_space
        self.action_space = env.action_space

    def reset(self, seed=None):
        o, info = self.env.reset(seed=seed)
        return np.asarray(o)[None], info

    def step(self, a):
        o, r, te, tr, info = self.env.step(a[0])
        o = np.asarray(o)[None]
        final = o
        if te or tr:
            o, _ = self.env.reset()
            o = np.asarray(o)[None]
        return o, np.asarray([r], dtype=np.float32), np.asarray([te]), np.asarray([tr]), {"final_obs": final}


_MA_REGISTRY: Dict[str, Callable] = {}


def register_multi_agent_env(name: str, creator: Callable):
    _MA_REGISTRY[name] = creator


def make_multi_agent_env(spec, config: Optional[dict] = None) -> MultiAgentEnv:
    if isinstance(spec, MultiAgentEnv):
        return spec
    if isinstance(spec, str):
        if spec in _MA_REGISTRY:
            return _MA_REGISTRY[spec](dict(config or {}))
        from .envs import _REGISTRY

        if spec in _REGISTRY:
            env = _REGISTRY[spec](dict(config or {}))
            if isinstance(env, MultiAgentEnv):
                return env
        raise ValueError(f"{spec!r} is not a registered multi-agent env")
    if isinstance(spec, type) and issubclass(spec, MultiAgentEnv):
        return spec(dict(config or {})) if _takes_config(spec) else spec()
    if callable(spec):
        env = spec(dict(config or {}))
        if isinstance(env, MultiAgentEnv):
            return env
    raise ValueError(f"cannot build a multi-agent env from {spec!r}")


def _takes_config(cls):
    import inspect

    try:
        return len(inspect.signature(cls.__init__).parameters) > 1
    except (TypeError, ValueError):
        return False


register_multi_agent_env("MultiAgentCartPole", make_multi_agent("CartPole-v1"))
