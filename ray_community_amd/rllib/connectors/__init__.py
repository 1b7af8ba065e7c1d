"""ConnectorV2 data pipelines (reference: ``rllib/connectors/``). See ``connector_v2.py``."""
from __future__ import annotations

from typing import Dict

from .connector_v2 import (ConnectorPipelineV2, ConnectorV2, EnvToModulePipeline, LearnerConnectorPipeline,
                           ModuleToEnvPipeline, VectorEnvContext)
from .env_to_module import FlattenObservations, FrameStackingEnvToModule, MeanStdFilter, PrevActionsPrevRewards
from .learner import ClipRewards, GeneralAdvantageEstimation
from .module_to_env import ClipActions, NormalizeAndClipActions


def _as_list(x):
    if x is None:
        return []
    if isinstance(x, ConnectorPipelineV2):
        return list(x.connectors)
    if isinstance(x, (list, tuple)):
        return list(x)
    return [x]


def build_env_to_module(config: Dict, env) -> EnvToModulePipeline:
    """User pieces from ``config["env_to_module_connector"](env)`` (a connector, a list of them
    or a pipeline), then the defaults the model config asks for: previous actions / rewards
    when ``lstm_use_prev_action`` / ``lstm_use_prev_reward`` are set (reference default
    pipeline)."""
    fn = config.get("env_to_module_connector")
    pieces = _as_list(fn(env) if callable(fn) else fn)
    m = config.get("model") or {}
    if config.get("add_default_connectors_to_env_to_module_pipeline", True) and \
            (m.get("lstm_use_prev_action") or m.get("lstm_use_prev_reward")):
        pieces.append(PrevActionsPrevRewards(n_prev_actions=int(bool(m.get("lstm_use_prev_action"))),
                                             n_prev_rewards=int(bool(m.get("lstm_use_prev_reward")))))
    return EnvToModulePipeline(env.observation_space, env.action_space, connectors=pieces)


def build_module_to_env(config: Dict, env) -> ModuleToEnvPipeline:
    fn = config.get("module_to_env_connector")
    pieces = _as_list(fn(env) if callable(fn) else fn)
    if config.get("normalize_actions") or config.get("clip_actions"):
        pieces.append(NormalizeAndClipActions(normalize_actions=bool(config.get("normalize_actions")),
                                              clip_actions=bool(config.get("clip_actions"))))
    return ModuleToEnvPipeline(env.observation_space, env.action_space, connectors=pieces)


def build_learner_connector(config: Dict, obs_space, act_space) -> LearnerConnectorPipeline:
    fn = config.get("learner_connector")
    pieces = _as_list(fn(obs_space, act_space) if callable(fn) else fn)
    return LearnerConnectorPipeline(obs_space, act_space, connectors=pieces)


__all__ = ["ConnectorV2", "ConnectorPipelineV2", "EnvToModulePipeline", "ModuleToEnvPipeline",
           "LearnerConnectorPipeline", "VectorEnvContext", "FlattenObservations", "MeanStdFilter",
           "PrevActionsPrevRewards", "FrameStackingEnvToModule", "NormalizeAndClipActions", "ClipActions",
           "GeneralAdvantageEstimation", "ClipRewards", "build_env_to_module", "build_module_to_env",
           "build_learner_connector"]
