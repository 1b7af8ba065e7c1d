"""Env wrappers for third-party simulators (reference: rllib/env/wrappers/*,
rllib/env/{dm_env,pettingzoo_env,...}) and ``RemoteBaseEnv`` (rllib/env/remote_base_env.py).

DeepMind dm_env / dm_control, PettingZoo and Unity ML-Agents are not installed in this
environment: their wrappers raise ImportError when constructed, naming the missing package.
``RemoteBaseEnv`` steps each sub-environment inside its own actor and polls whichever ones
have finished a step, so slow simulators overlap."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

from ..external_env import BaseEnv


class _NeedsPackage:
    _PKG = ""

    def __init__(self, *a, **k):
        raise ImportError(f"{type(self).__name__} needs `{self._PKG}`, which is not installed in this environment")


class DMEnv(_NeedsPackage):
    _PKG = "dm_env"


class DMCEnv(_NeedsPackage):
    _PKG = "dm_control"


class PettingZooEnv(_NeedsPackage):
    _PKG = "pettingzoo"


class ParallelPettingZooEnv(_NeedsPackage):
    _PKG = "pettingzoo"


class Unity3DEnv(_NeedsPackage):
    _PKG = "mlagents_envs"


class _EnvActor:
    def __init__(self, make_env: Callable[[int], Any], index: int):
        self.env = make_env(index)

    def reset(self):
        out = self.env.reset()
        return out if isinstance(out, tuple) else (out, {})

    def step(self, action):
        return self.env.step(action)


class RemoteBaseEnv(BaseEnv):
    """``num_envs`` copies of ``make_env(index)`` in actors. ``poll`` returns the sub-envs whose
    reset / step finished (all of them when ``remote_env_batch_wait_ms`` is 0, else whatever is
    ready within that many ms, at least one), keyed by sub-env index."""

    def __init__(self, make_env: Callable[[int], Any], num_envs: int, remote_env_batch_wait_ms: int = 0,
                 restart_failed_sub_environments: bool = False):
        from .... import remote

        self.make_env, self.num_envs = make_env, int(num_envs)
        self.wait_ms = int(remote_env_batch_wait_ms)
        self._cls = remote(num_cpus=0)(_EnvActor)
        self.actors = [self._cls.remote(make_env, i) for i in range(self.num_envs)]
        self._pending: Dict[Any, int] = {a.reset.remote(): i for i, a in enumerate(self.actors)}
        self._resetting = set(range(self.num_envs))

    def poll(self):
        from .... import get, wait

        refs = list(self._pending)
        if not refs:
            return {}, {}, {}, {}, {}, {}
        if self.wait_ms == 0:
            ready = refs
        else:
            ready, _ = wait(refs, num_returns=1)
            more, _ = wait([r for r in refs if r not in ready], num_returns=len(refs) - len(ready),
                           timeout=self.wait_ms / 1000.0) if len(refs) > len(ready) else ([], [])
            ready = list(ready) + list(more)
        obs, rew, term, trunc, infos = {}, {}, {}, {}, {}
        for r in ready:
            i = self._pending.pop(r)
            out = get(r)
            if i in self._resetting:
                self._resetting.discard(i)
                obs[i], infos[i] = out
                rew[i], term[i], trunc[i] = 0.0, False, False
            else:
                obs[i], rew[i], term[i], trunc[i], infos[i] = out
        term["__all__"] = False
        trunc["__all__"] = False
        return obs, rew, term, trunc, infos, {}

    def send_actions(self, action_dict: Dict[int, Any]) -> None:
        for i, a in action_dict.items():
            self._pending[self.actors[i].step.remote(a)] = i

    def try_reset(self, env_id: Optional[int] = None):
        ids = range(self.num_envs) if env_id is None else [env_id]
        for i in ids:
            self._resetting.add(i)
            self._pending[self.actors[i].reset.remote()] = i
        return None

    def get_sub_environments(self) -> List[Any]:
        return list(self.actors)

    def stop(self):
        from .... import kill

        for a in self.actors:
            try:
                kill(a)
            except Exception:
                pass
