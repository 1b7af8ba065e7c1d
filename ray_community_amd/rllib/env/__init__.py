from .base_env import convert_to_base_env
from .env_context import EnvContext
from .env_runner import EnvRunner
from .envs import CartPoleVec, Env, PendulumVec, SyntheticAtariVec, VectorEnv, make_vector_env, register_env
from .external_env import BaseEnv, ExternalEnv, ExternalMultiAgentEnv
from .multi_agent_env import MultiAgentEnv, _GroupedAgents as GroupAgentsWrapper, make_multi_agent, \
    register_multi_agent_env
from .multi_agent_env_runner import MultiAgentEnvRunner
from .policy_client import PolicyClient
from .policy_server_input import PolicyServerInput
from .wrappers import DMCEnv, DMEnv, ParallelPettingZooEnv, PettingZooEnv, RemoteBaseEnv, Unity3DEnv

__all__ = ["Env", "VectorEnv", "CartPoleVec", "PendulumVec", "SyntheticAtariVec", "make_vector_env", "register_env",
           "EnvRunner", "MultiAgentEnv", "make_multi_agent", "register_multi_agent_env", "MultiAgentEnvRunner",
           "BaseEnv", "EnvContext", "ExternalEnv", "ExternalMultiAgentEnv", "GroupAgentsWrapper", "PolicyClient",
           "PolicyServerInput", "RemoteBaseEnv", "DMEnv", "DMCEnv", "PettingZooEnv", "ParallelPettingZooEnv",
           "Unity3DEnv", "convert_to_base_env"]
