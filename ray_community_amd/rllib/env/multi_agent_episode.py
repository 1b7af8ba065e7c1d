"""MultiAgentEpisode: one multi-agent env episode as per-agent SingleAgentEpisodes (reference:
``rllib/env/multi_agent_episode.py:32``).

Agents may act asynchronously: an agent's env step (obs, action, reward, next obs) is recorded
when it receives its NEXT observation. Between its action and that observation its rewards are
"hanging" and summed; an agent that terminates (or the episode, ``"__all__"``) closes its
transition with the reward collected so far. ``env_t`` counts env steps of the whole episode,
each agent episode its own agent steps. ``agent_to_module_mapping_fn`` names the module (policy)
of every agent, used by ``to_sample_batch`` (one SampleBatch per module).
"""
from __future__ import annotations

import uuid
from typing import Any, Callable, Dict, Optional

import numpy as np

from .single_agent_episode import SingleAgentEpisode

ALL = "__all__"


class MultiAgentEpisode:
    def __init__(self, id_: Optional[str] = None, *, agent_to_module_mapping_fn: Optional[Callable] = None,
                 env_t_started: int = 0):
        self.id_ = id_ or uuid.uuid4().hex
        self.agent_to_module_mapping_fn = agent_to_module_mapping_fn or (lambda aid, ep=None: "default_policy")
        self.agent_episodes: Dict[Any, SingleAgentEpisode] = {}
        self.env_t_started = int(env_t_started)
        self.env_t = self.env_t_started
        self.is_terminated = False
        self.is_truncated = False
        self._hanging_action: Dict[Any, Any] = {}
        self._hanging_reward: Dict[Any, float] = {}
        self._hanging_extra: Dict[Any, Dict] = {}
        self._module_for: Dict[Any, Any] = {}
        self._last_stepped = set()

    # ------------------------------------------------------------------ building
    def module_for(self, agent_id):
        m = self._module_for.get(agent_id)
        if m is None:
            m = self._module_for[agent_id] = self.agent_to_module_mapping_fn(agent_id, self)
        return m

    def _agent_episode(self, agent_id) -> SingleAgentEpisode:
        ep = self.agent_episodes.get(agent_id)
        if ep is None:
            ep = self.agent_episodes[agent_id] = SingleAgentEpisode(
                agent_id=agent_id, module_id=self.module_for(agent_id), multi_agent_episode_id=self.id_)
        return ep

    def add_env_reset(self, observations: Dict, infos: Optional[Dict] = None):
        infos = infos or {}
        for aid, o in observations.items():
            self._agent_episode(aid).add_env_reset(o, infos.get(aid))
        self._last_stepped = set(observations)

    def add_env_step(self, observations: Dict, actions: Dict, rewards: Dict, infos: Optional[Dict] = None, *,
                     terminateds: Optional[Dict] = None, truncateds: Optional[Dict] = None,
                     extra_model_outputs: Optional[Dict[Any, Dict]] = None):
        """One env step: ``actions`` are what the acting agents sent (on their previous
        observations), the rest is what ``env.step`` returned."""
        infos, terminateds, truncateds = infos or {}, terminateds or {}, truncateds or {}
        extra_model_outputs = extra_model_outputs or {}
        for aid, a in actions.items():
            self._hanging_action[aid] = a
            self._hanging_reward.setdefault(aid, 0.0)
            self._hanging_extra[aid] = dict(extra_model_outputs.get(aid) or {})
        for aid, r in rewards.items():
            if aid in self._hanging_action:
                self._hanging_reward[aid] = self._hanging_reward.get(aid, 0.0) + float(r)
        all_term = bool(terminateds.get(ALL, False))
        all_trunc = bool(truncateds.get(ALL, False))
        for aid, ep in list(self.agent_episodes.items()) + [(a, None) for a in observations
                                                             if a not in self.agent_episodes]:
            if ep is not None and ep.is_done:
                continue
            term = bool(terminateds.get(aid, False)) or all_term
            trunc = (bool(truncateds.get(aid, False)) or all_trunc) and not term
            if aid in observations:
                if aid in self._hanging_action:
                    self._agent_episode(aid).add_env_step(
                        observations[aid], self._hanging_action.pop(aid), self._hanging_reward.pop(aid),
                        infos.get(aid), terminated=term, truncated=trunc,
                        extra_model_outputs=self._hanging_extra.pop(aid, None))
                elif ep is None or not ep.is_reset:
                    self._agent_episode(aid).add_env_reset(observations[aid], infos.get(aid))
            elif (term or trunc) and aid in self._hanging_action:
                # done without a final observation: close the transition on its last one
                last = self._agent_episode(aid).get_observations(-1)
                self._agent_episode(aid).add_env_step(
                    last, self._hanging_action.pop(aid), self._hanging_reward.pop(aid), infos.get(aid),
                    terminated=term, truncated=trunc, extra_model_outputs=self._hanging_extra.pop(aid, None))
        self.env_t += 1
        self._last_stepped = set(observations)
        self.is_terminated = all_term or (bool(self.agent_episodes) and all(
            e.is_terminated for e in self.agent_episodes.values()))
        self.is_truncated = (all_trunc and not self.is_terminated)

    def finalize(self) -> "MultiAgentEpisode":
        for ep in self.agent_episodes.values():
            ep.finalize()
        return self

    # ------------------------------------------------------------------ access
    @property
    def is_done(self) -> bool:
        return self.is_terminated or self.is_truncated

    @property
    def agent_ids(self):
        return set(self.agent_episodes)

    def __len__(self) -> int:
        return self.env_t - self.env_t_started

    def env_steps(self) -> int:
        return len(self)

    def agent_steps(self) -> int:
        return sum(len(e) for e in self.agent_episodes.values())

    def get_return(self, include_hanging_rewards: bool = False) -> float:
        r = sum(e.get_return() for e in self.agent_episodes.values())
        if include_hanging_rewards:
            r += sum(self._hanging_reward.values())
        return float(r)

    def get_agents_to_act(self):
        """Agents whose latest observation is not yet answered by an action."""
        return {aid for aid, e in self.agent_episodes.items() if not e.is_done and aid not in self._hanging_action
                and e.is_reset}

    def get_observations(self, indices=-1, agent_ids=None, **kw) -> Dict:
        ids = self.agent_episodes if agent_ids is None else agent_ids
        return {aid: self.agent_episodes[aid].get_observations(indices, **kw) for aid in ids
                if aid in self.agent_episodes and self.agent_episodes[aid].is_reset}

    def get_actions(self, indices=-1, agent_ids=None, **kw) -> Dict:
        ids = self.agent_episodes if agent_ids is None else agent_ids
        return {aid: self.agent_episodes[aid].get_actions(indices, **kw) for aid in ids
                if aid in self.agent_episodes and len(self.agent_episodes[aid].actions)}

    def get_rewards(self, indices=-1, agent_ids=None, **kw) -> Dict:
        ids = self.agent_episodes if agent_ids is None else agent_ids
        return {aid: self.agent_episodes[aid].get_rewards(indices, **kw) for aid in ids
                if aid in self.agent_episodes and len(self.agent_episodes[aid].rewards)}

    def get_infos(self, indices=-1, agent_ids=None, **kw) -> Dict:
        ids = self.agent_episodes if agent_ids is None else agent_ids
        return {aid: self.agent_episodes[aid].get_infos(indices, **kw) for aid in ids
                if aid in self.agent_episodes and self.agent_episodes[aid].is_reset}

    def get_extra_model_outputs(self, key: str, indices=-1, agent_ids=None, **kw) -> Dict:
        ids = self.agent_episodes if agent_ids is None else agent_ids
        return {aid: self.agent_episodes[aid].get_extra_model_outputs(key, indices, **kw) for aid in ids
                if aid in self.agent_episodes and key in self.agent_episodes[aid].extra_model_outputs
                and len(self.agent_episodes[aid].extra_model_outputs[key])}

    def get_terminateds(self) -> Dict:
        out = {aid: e.is_terminated for aid, e in self.agent_episodes.items()}
        out["__all__"] = self.is_terminated
        return out

    def get_truncateds(self) -> Dict:
        out = {aid: e.is_truncated for aid, e in self.agent_episodes.items()}
        out["__all__"] = self.is_truncated
        return out

    @property
    def agent_episode_ids(self) -> Dict:
        return {aid: e.id_ for aid, e in self.agent_episodes.items()}

    @property
    def is_finalized(self) -> bool:
        return bool(self.agent_episodes) and all(e.is_finalized for e in self.agent_episodes.values())

    def get_agents_that_stepped(self):
        """Agents that received an observation at the latest reset / env step."""
        return set(self._last_stepped)

    def validate(self) -> None:
        for aid, e in self.agent_episodes.items():
            e.validate()
            if e.multi_agent_episode_id not in (None, self.id_):
                raise AssertionError(f"agent {aid}'s episode belongs to {e.multi_agent_episode_id}")

    def get_sample_batch(self):
        return self.to_sample_batch()

    # ------------------------------------------------------------------ chunks / conversion
    def cut(self, len_lookback_buffer: int = 0) -> "MultiAgentEpisode":
        nxt = MultiAgentEpisode(self.id_, agent_to_module_mapping_fn=self.agent_to_module_mapping_fn,
                                env_t_started=self.env_t)
        nxt._module_for = dict(self._module_for)
        nxt._last_stepped = set(self._last_stepped)
        for aid, ep in self.agent_episodes.items():
            if not ep.is_done:
                nxt.agent_episodes[aid] = ep.cut(len_lookback_buffer)
        nxt._hanging_action = dict(self._hanging_action)
        nxt._hanging_reward = dict(self._hanging_reward)
        nxt._hanging_extra = dict(self._hanging_extra)
        return nxt

    def to_sample_batch(self):
        """MultiAgentBatch: per module, the concatenated transitions of its agents."""
        from ..policy.sample_batch import MultiAgentBatch, SampleBatch, concat_samples

        per = {}
        for aid, ep in self.agent_episodes.items():
            if len(ep):
                b = ep.to_sample_batch()
                b["agent_index"] = np.full(b.count, hash(aid) & 0x7FFF, dtype=np.int64)
                per.setdefault(self.module_for(aid), []).append(b)
        return MultiAgentBatch({m: concat_samples(bs) if len(bs) > 1 else bs[0] for m, bs in per.items()},
                               env_steps=len(self))

    def get_state(self) -> Dict:
        return {"id_": self.id_, "env_t_started": self.env_t_started, "env_t": self.env_t,
                "terminated": self.is_terminated, "truncated": self.is_truncated,
                "agent_episodes": {aid: e.get_state() for aid, e in self.agent_episodes.items()},
                "hanging": (dict(self._hanging_action), dict(self._hanging_reward), dict(self._hanging_extra)),
                "modules": dict(self._module_for)}

    @staticmethod
    def from_state(state: Dict, agent_to_module_mapping_fn=None) -> "MultiAgentEpisode":
        ep = MultiAgentEpisode(state["id_"], agent_to_module_mapping_fn=agent_to_module_mapping_fn,
                               env_t_started=state["env_t_started"])
        ep.env_t = state["env_t"]
        ep.is_terminated, ep.is_truncated = state["terminated"], state["truncated"]
        ep.agent_episodes = {aid: SingleAgentEpisode.from_state(s) for aid, s in state["agent_episodes"].items()}
        ep._hanging_action, ep._hanging_reward, ep._hanging_extra = (dict(x) for x in state["hanging"])
        ep._module_for = dict(state["modules"])
        return ep

    def __repr__(self):
        return f"MAEps(len={len(self)} done={self.is_done} agents={sorted(map(str, self.agent_ids))} id_={self.id_[:8]})"
