"""ConnectorV2 and connector pipelines (reference: ``rllib/connectors/connector_v2.py``,
``connector_pipeline_v2.py``, ``env_to_module/env_to_module_pipeline.py``,
``module_to_env/module_to_env_pipeline.py``, ``learner/learner_connector_pipeline.py``).

A connector is a callable piece that transforms a batch on one of the three data paths:

  * env -> module (in the env runner, every env step): raw env observations of the N
    vectorised sub-envs -> the RLModule's input (``batch["obs"]``, numpy ``[N, ...]``);
  * module -> env (in the env runner): the module's sampled actions -> the actions the env
    steps with (``batch["actions_for_env"]``; ``batch["actions"]`` stays what the loss sees);
  * learner (in the learner, once per update): the env-major ``[N, T]`` train batch, already
    resident on the learner's device (torch tensors), before the loss.

The runner here is vectorised (one numpy batch for N sub-envs, no per-episode Python objects), so
the "episodes" argument is a :class:`VectorEnvContext`: per-env ``is_first`` flags (an episode
starts at this observation), the previous step's actions and rewards. Stateful connectors keep
per-env history rows and reset the rows whose ``is_first`` is set. ``shared_data["peek"]``
asks a stateful connector for its output WITHOUT committing a state update (the runner uses it
for the final observation of truncated episodes, whose value bootstraps GAE).

Connector state (e.g. running observation statistics) is collected from every env runner,
merged with ``merge_states`` and broadcast back by the Algorithm once per iteration.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Union

import numpy as np


class VectorEnvContext:
    """What the vectorised runner knows about the N sub-envs' episodes at one env step."""

    def __init__(self, num_envs: int):
        self.num_envs = num_envs
        self.is_first = np.ones(num_envs, dtype=bool)
        self.last_actions: Optional[np.ndarray] = None
        self.last_rewards = np.zeros(num_envs, dtype=np.float32)
        self.env_indices: Optional[np.ndarray] = None  # rows of a partial (peek) batch

    def subset(self, idx, actions, rewards) -> "VectorEnvContext":
        c = VectorEnvContext(len(idx))
        c.is_first = np.zeros(len(idx), dtype=bool)
        c.last_actions = None if actions is None else np.asarray(actions)[idx]
        c.last_rewards = np.asarray(rewards, dtype=np.float32)[idx]
        c.env_indices = np.asarray(idx)
        return c


class ConnectorV2:
    def __init__(self, input_observation_space=None, input_action_space=None, **kwargs):
        self._input_observation_space = None
        self._input_action_space = None
        self._observation_space = None
        self._action_space = None
        if input_observation_space is not None or input_action_space is not None:
            self.set_input_spaces(input_observation_space, input_action_space)

    # ------------------------------------------------------------------ spaces
    def set_input_spaces(self, observation_space, action_space):
        self._input_observation_space = observation_space
        self._input_action_space = action_space
        self._observation_space = self.recompute_output_observation_space(observation_space, action_space)
        self._action_space = self.recompute_output_action_space(observation_space, action_space)

    @property
    def input_observation_space(self):
        return self._input_observation_space

    @input_observation_space.setter
    def input_observation_space(self, s):
        self.set_input_spaces(s, self._input_action_space)

    @property
    def input_action_space(self):
        return self._input_action_space

    @input_action_space.setter
    def input_action_space(self, s):
        self.set_input_spaces(self._input_observation_space, s)

    @property
    def observation_space(self):
        return self._observation_space if self._observation_space is not None else self._input_observation_space

    @property
    def action_space(self):
        return self._action_space if self._action_space is not None else self._input_action_space

    def recompute_output_observation_space(self, input_observation_space, input_action_space):
        return input_observation_space

    def recompute_output_action_space(self, input_observation_space, input_action_space):
        return input_action_space

    # ------------------------------------------------------------------ call / state
    def __call__(self, *, rl_module=None, batch: Dict[str, Any], episodes=None, explore: Optional[bool] = None,
                 shared_data: Optional[dict] = None, metrics=None, **kwargs) -> Dict[str, Any]:
        raise NotImplementedError

    def get_state(self, components=None, *, not_components=None, **kwargs) -> Dict[str, Any]:
        return {}

    def set_state(self, state: Dict[str, Any]) -> None:
        pass

    def reset_state(self) -> None:
        pass

    @staticmethod
    def merge_states(states: List[Dict[str, Any]]) -> Dict[str, Any]:
        return states[0] if states else {}

    @property
    def name(self) -> str:
        return type(self).__name__

    def __repr__(self):
        return f"{self.name}()"


def _matches(c: ConnectorV2, key) -> bool:
    if isinstance(key, str):
        return c.name == key
    if isinstance(key, type):
        return isinstance(c, key)
    return c is key


class ConnectorPipelineV2(ConnectorV2):
    """An ordered list of connectors run one after the other; the output spaces of each piece
    are the input spaces of the next."""

    def __init__(self, input_observation_space=None, input_action_space=None, *,
                 connectors: Optional[Sequence[ConnectorV2]] = None, **kwargs):
        self.connectors: List[ConnectorV2] = list(connectors or [])
        super().__init__(input_observation_space, input_action_space, **kwargs)

    def _respace(self):
        obs, act = self._input_observation_space, self._input_action_space
        for c in self.connectors:
            c.set_input_spaces(obs, act)
            obs, act = c.observation_space, c.action_space
        self._observation_space, self._action_space = obs, act

    def set_input_spaces(self, observation_space, action_space):
        self._input_observation_space = observation_space
        self._input_action_space = action_space
        self._respace()

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=None, shared_data=None, metrics=None,
                 **kwargs):
        shared_data = {} if shared_data is None else shared_data
        for c in self.connectors:
            batch = c(rl_module=rl_module, batch=batch, episodes=episodes, explore=explore, shared_data=shared_data,
                      metrics=metrics, **kwargs)
            if batch is None:
                raise ValueError(f"connector {c.name} returned None (must return the batch)")
        return batch

    # ------------------------------------------------------------------ editing
    def _index(self, key) -> int:
        for i, c in enumerate(self.connectors):
            if _matches(c, key):
                return i
        raise ValueError(f"no connector {key!r} in {self}")

    def append(self, connector: ConnectorV2):
        self.connectors.append(connector)
        self._respace()
        return connector

    def prepend(self, connector: ConnectorV2):
        self.connectors.insert(0, connector)
        self._respace()
        return connector

    def insert_before(self, key, connector: ConnectorV2):
        self.connectors.insert(self._index(key), connector)
        self._respace()
        return connector

    def insert_after(self, key, connector: ConnectorV2):
        self.connectors.insert(self._index(key) + 1, connector)
        self._respace()
        return connector

    def remove(self, key):
        self.connectors.pop(self._index(key))
        self._respace()

    def __len__(self):
        return len(self.connectors)

    def __getitem__(self, key) -> Union[ConnectorV2, List[ConnectorV2]]:
        if isinstance(key, (int, slice)):
            return self.connectors[key]
        found = [c for c in self.connectors if _matches(c, key)]
        if not found:
            raise KeyError(key)
        return found

    # ------------------------------------------------------------------ state
    def _keys(self):
        return [f"{i:03d}_{c.name}" for i, c in enumerate(self.connectors)]

    def get_state(self, components=None, *, not_components=None, **kwargs):
        return {k: c.get_state() for k, c in zip(self._keys(), self.connectors)}

    def set_state(self, state):
        for k, c in zip(self._keys(), self.connectors):
            if k in state:
                c.set_state(state[k])

    def reset_state(self):
        for c in self.connectors:
            c.reset_state()

    def merge_states(self, states: List[Dict[str, Any]]) -> Dict[str, Any]:  # noqa: D401 - instance method here
        return {k: c.merge_states([s[k] for s in states if k in s]) for k, c in zip(self._keys(), self.connectors)}

    def __repr__(self):
        return f"{type(self).__name__}({', '.join(c.name for c in self.connectors)})"


class EnvToModulePipeline(ConnectorPipelineV2):
    pass


class ModuleToEnvPipeline(ConnectorPipelineV2):
    pass


class LearnerConnectorPipeline(ConnectorPipelineV2):
    pass
