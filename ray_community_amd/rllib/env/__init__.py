from .envs import CartPoleVec, Env, PendulumVec, SyntheticAtariVec, VectorEnv, make_vector_env, register_env
from .env_runner import EnvRunner
from .multi_agent_env import MultiAgentEnv, make_multi_agent, register_multi_agent_env
from .multi_agent_env_runner import MultiAgentEnvRunner

__all__ = ["Env", "VectorEnv", "CartPoleVec", "PendulumVec", "SyntheticAtariVec", "make_vector_env", "register_env",
           "EnvRunner", "MultiAgentEnv", "make_multi_agent", "register_multi_agent_env", "MultiAgentEnvRunner"]
