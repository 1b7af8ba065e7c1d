"""Type aliases used in RLlib signatures (reference: ``rllib/utils/typing.py``), for user code that
annotates custom envs, modules, learners and callbacks with them. They are plain ``typing``
aliases: nothing here is checked at run time."""
from __future__ import annotations

from typing import Any, Callable, Dict, Hashable, List, Optional, Tuple, TypeVar, Union

import numpy as np

try:  # torch is the only tensor framework here
    import torch

    TensorType = Union[np.ndarray, "torch.Tensor"]
except ImportError:  # pragma: no cover
    TensorType = np.ndarray

TensorStructType = Union[TensorType, dict, tuple]
TensorShape = Union[Tuple[int, ...], List[int]]
NetworkType = Any  # a torch.nn.Module
AlgorithmConfigDict = Dict[str, Any]
PartialAlgorithmConfigDict = Dict[str, Any]
ModelConfigDict = Dict[str, Any]
FromConfigSpec = Union[Dict[str, Any], type, str]
EnvConfigDict = Dict[str, Any]
EnvID = Union[int, str]
EnvType = Any  # a gym-style env, MultiAgentEnv, VectorEnv or BaseEnv
EnvCreator = Callable[[EnvConfigDict], Optional[EnvType]]
AgentID = Hashable
PolicyID = str
ModuleID = str
MultiAgentPolicyConfigDict = Dict[PolicyID, Any]
EpisodeType = Any  # SingleAgentEpisode or MultiAgentEpisode
IsPolicyToTrain = Callable[[PolicyID, Optional[Any]], bool]
AgentToModuleMappingFn = Callable[[AgentID, EpisodeType], ModuleID]
ShouldModuleBeUpdatedFn = Union[List[ModuleID], Callable[[ModuleID, Optional[Any]], bool]]
PolicyState = Dict[str, TensorStructType]
EpisodeID = Union[int, str]
UnrollID = int
MultiAgentDict = Dict[AgentID, Any]
MultiEnvDict = Dict[EnvID, MultiAgentDict]
EnvObsType = Any
EnvActionType = Any
EnvInfoDict = dict
FileType = Any
ViewRequirementsDict = Dict[str, Any]
ResultDict = dict
LocalOptimizer = Any  # a torch.optim.Optimizer
Optimizer = Any
Param = Any  # a torch.nn.Parameter
ParamRef = Hashable
ParamDict = Dict[ParamRef, Param]
LearningRateOrSchedule = Union[float, List[List[Union[int, float]]], List[Tuple[int, Union[int, float]]]]
GradInfoDict = dict
LearnerStatsDict = dict
ModelGradients = Union[List[Tuple[TensorType, TensorType]], List[TensorType]]
ModelWeights = dict
ModelInputDict = Dict[str, TensorType]
SampleBatchType = Any  # SampleBatch or MultiAgentBatch
SpaceStruct = Any
StateBatches = List[List[Any]]
PolicyOutputType = Tuple[TensorStructType, StateBatches, Dict[str, TensorType]]
T = TypeVar("T")
