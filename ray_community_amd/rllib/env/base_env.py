"""BaseEnv conversion (reference ``rllib/env/base_env.py`` ``convert_to_base_env``): any env as
the async multi-env interface -- ``poll()`` returns ``{env_id: {agent_id: value}}`` dicts for the
sub-environments that have new data, ``send_actions({env_id: {agent_id: action}})`` steps them."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

from .external_env import BaseEnv, ExternalEnv
from .multi_agent_env import MultiAgentEnv

_SINGLE = "agent0"


class _MultiEnvBase(BaseEnv):
    def __init__(self, envs: List[Any], multi_agent: bool):
        self.envs = envs
        self.multi_agent = multi_agent
        self._pending: Dict[int, tuple] = {}
        for i in range(len(envs)):
            self._reset(i)

    def _wrap(self, d):
        return d if self.multi_agent else {_SINGLE: d}

    def _reset(self, i):
        obs, info = self.envs[i].reset()
        self._pending[i] = (self._wrap(obs), {}, {"__all__": False}, {"__all__": False}, self._wrap(info))

    def poll(self):
        obs, rew, term, trunc, infos = {}, {}, {}, {}, {}
        for i, (o, r, te, tr, inf) in list(self._pending.items()):
            obs[i], rew[i], term[i], trunc[i], infos[i] = o, r, te, tr, inf
        self._pending.clear()
        return obs, rew, term, trunc, infos, {}

    def send_actions(self, action_dict: Dict[int, Dict]) -> None:
        for i, acts in action_dict.items():
            env = self.envs[i]
            if self.multi_agent:
                o, r, te, tr, inf = env.step(acts)
            else:
                o1, r1, te1, tr1, inf1 = env.step(acts[_SINGLE])
                o, r, inf = {_SINGLE: o1}, {_SINGLE: r1}, {_SINGLE: inf1}
                te = {_SINGLE: te1, "__all__": bool(te1)}
                tr = {_SINGLE: tr1, "__all__": bool(tr1)}
            self._pending[i] = (o, r, te, tr, inf)

    def try_reset(self, env_id: Optional[int] = None):
        ids = range(len(self.envs)) if env_id is None else [env_id]
        out = {}
        for i in ids:
            self._reset(i)
            out[i] = self._pending[i][0]
        return out, {i: self._pending[i][4] for i in ids}

    def get_sub_environments(self):
        return list(self.envs)

    def stop(self):
        for e in self.envs:
            if hasattr(e, "close"):
                e.close()


def convert_to_base_env(env, make_env: Optional[Callable[[int], Any]] = None, num_envs: int = 1,
                        remote_envs: bool = False, remote_env_batch_wait_ms: int = 0,
                        worker=None, restart_failed_sub_environments: bool = False) -> BaseEnv:
    if isinstance(env, BaseEnv):
        return env
    if isinstance(env, ExternalEnv):
        return env.to_base_env()
    envs = [env] + [make_env(i) for i in range(1, num_envs)] if (make_env and num_envs > 1) else [env]
    return _MultiEnvBase(envs, multi_agent=isinstance(env, MultiAgentEnv))
