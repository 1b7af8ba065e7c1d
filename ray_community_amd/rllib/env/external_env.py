"""Environments that drive the agent instead of being stepped by it (reference
``rllib/env/external_env.py``, ``rllib/env/base_env.py``).

``ExternalEnv.run()`` executes in its own thread and talks to the policy through
``start_episode`` / ``get_action`` / ``log_action`` / ``log_returns`` / ``end_episode``; the sampler
side sees it as a ``BaseEnv``: ``poll()`` returns the observations that wait for actions (and the
rewards / dones logged since the last poll), ``send_actions`` answers them.
"""
from __future__ import annotations

import queue
import threading
import uuid
from typing import Any, Dict, Optional, Tuple


class BaseEnv:
    """Async, multi-episode env interface: ``poll() -> (obs, rewards, terminateds, truncateds,
    infos, off_policy_actions)`` keyed by episode id, ``send_actions({episode_id: action})``."""

    def poll(self) -> Tuple[Dict, Dict, Dict, Dict, Dict, Dict]:
        raise NotImplementedError

    def send_actions(self, action_dict: Dict[str, Any]) -> None:
        raise NotImplementedError

    def try_reset(self, env_id: Optional[str] = None):
        return None

    def get_sub_environments(self):
        return []

    def stop(self):
        pass


class _Episode:
    def __init__(self, eid, training_enabled):
        self.eid = eid
        self.training_enabled = training_enabled
        self.reward = 0.0
        self.done = False
        self.action_q: "queue.Queue" = queue.Queue(maxsize=1)
        self.pending_obs = None
        self.logged_action = None


class ExternalEnv(threading.Thread):
    def __init__(self, action_space, observation_space, max_concurrent: int = 100):
        super().__init__(daemon=True)
        self.action_space = action_space
        self.observation_space = observation_space
        self.max_concurrent = max_concurrent
        self._episodes: Dict[str, _Episode] = {}
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        self._finished: Dict[str, float] = {}

    def run(self):
        """Override: the env's main loop (usually serving requests)."""
        raise NotImplementedError

    # -------------------------------------------------------------- env-side API
    def start_episode(self, episode_id: Optional[str] = None, training_enabled: bool = True) -> str:
        eid = episode_id or uuid.uuid4().hex
        with self._cv:
            if eid in self._episodes:
                raise ValueError(f"episode {eid} already started")
            if len(self._episodes) >= self.max_concurrent:
                raise ValueError(f"too many concurrent episodes (max_concurrent={self.max_concurrent})")
            self._episodes[eid] = _Episode(eid, training_enabled)
            self._episodes[eid].reward = self._zero_reward()
        return eid

    def get_action(self, episode_id: str, observation):
        ep = self._episodes[episode_id]
        with self._cv:
            ep.pending_obs = observation
            self._cv.notify_all()
        return ep.action_q.get()

    def log_action(self, episode_id: str, observation, action):
        ep = self._episodes[episode_id]
        with self._cv:
            ep.logged_action = (observation, action)
            self._cv.notify_all()

    def log_returns(self, episode_id: str, reward: float, info: Optional[Dict] = None):
        with self._cv:
            ep = self._episodes[episode_id]
            ep.reward = self._add_reward(ep.reward, reward)

    # reward accumulation between two polls: a float here, a per-agent dict in the multi-agent env
    def _zero_reward(self):
        return 0.0

    def _add_reward(self, acc, reward):
        return acc + float(reward)

    def end_episode(self, episode_id: str, observation):
        with self._cv:
            ep = self._episodes.pop(episode_id)
            ep.done = True
            self._finished[episode_id] = (observation, ep.reward)
            self._cv.notify_all()

    # -------------------------------------------------------------- sampler-side view
    def to_base_env(self) -> BaseEnv:
        return _ExternalBaseEnv(self)


class _ExternalBaseEnv(BaseEnv):
    def __init__(self, env: ExternalEnv):
        self.env = env
        if not env.is_alive():
            env.start()

    def poll(self, timeout: float = 60.0):
        env = self.env
        obs, rew, term, trunc, infos, off = {}, {}, {}, {}, {}, {}
        with env._cv:
            ok = env._cv.wait_for(lambda: env._finished or any(
                e.pending_obs is not None or e.logged_action is not None for e in env._episodes.values()), timeout)
            if not ok:
                return obs, rew, term, trunc, infos, off
            for eid, (o, r) in env._finished.items():
                obs[eid], rew[eid], term[eid], trunc[eid], infos[eid] = o, r, True, False, {}
            env._finished.clear()
            for eid, ep in env._episodes.items():
                if ep.pending_obs is not None:
                    obs[eid], rew[eid], term[eid], trunc[eid], infos[eid] = ep.pending_obs, ep.reward, False, False, {}
                    ep.reward = env._zero_reward()
                    ep.pending_obs = None
                elif ep.logged_action is not None:
                    o, a = ep.logged_action
                    obs[eid], rew[eid], term[eid], trunc[eid], infos[eid] = o, ep.reward, False, False, {}
                    off[eid] = a
                    ep.reward = env._zero_reward()
                    ep.logged_action = None
        return obs, rew, term, trunc, infos, off

    def send_actions(self, action_dict):
        for eid, a in action_dict.items():
            ep = self.env._episodes.get(eid)
            if ep is not None:
                ep.action_q.put(a)


class ExternalMultiAgentEnv(ExternalEnv):
    """Multi-agent external env (reference rllib/env/external_multi_agent_env.py): observations and
    actions are ``{agent_id: ...}`` dicts and ``log_returns`` takes ``{agent_id: reward}``, summed
    per agent until the next action request."""

    def _zero_reward(self):
        return {}

    def _add_reward(self, acc, reward):
        out = dict(acc)
        for aid, r in dict(reward).items():
            out[aid] = out.get(aid, 0.0) + float(r)
        return out
