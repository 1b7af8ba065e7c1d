from .envs import CartPoleVec, Env, PendulumVec, SyntheticAtariVec, VectorEnv, make_vector_env, register_env
from .env_runner import EnvRunner

__all__ = ["Env", "VectorEnv", "CartPoleVec", "PendulumVec", "SyntheticAtariVec", "make_vector_env", "register_env",
           "EnvRunner"]
