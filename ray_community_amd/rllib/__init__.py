"""RLlib equivalent (reference: ``rllib/``): PPO / DQN / IMPALA / APPO / SAC / CQL / MARWIL / BC,
vectorised env runners, GPU learners over RCCL, HIP GAE."""
from .algorithms import (APPO, BC, CQL, DQN, IMPALA, MARWIL, PPO, BCConfig, MARWILConfig, Algorithm, AlgorithmConfig, APPOConfig, DQNConfig, IMPALAConfig,
                         PPOConfig, SAC, SACConfig, CQLConfig, get_algorithm_class)
from .env import MultiAgentEnv, make_multi_agent, register_env
from .policy import PolicySpec
from .policy.policy import Policy, TFPolicy, TorchPolicy
from .env.envs import VectorEnv
from .env.external_env import BaseEnv, ExternalEnv
from .env.env_runner import EnvRunner as RolloutWorker  # old-stack name of the sampling actor
from .policy.sample_batch import MultiAgentBatch, SampleBatch

__all__ = ["PPO", "PPOConfig", "IMPALA", "IMPALAConfig", "APPO", "APPOConfig", "SAC", "SACConfig", "CQL", "CQLConfig", "MARWIL", "MARWILConfig", "BC", "BCConfig", "DQN", "DQNConfig", "Algorithm", "AlgorithmConfig", "SampleBatch", "MultiAgentBatch",
           "register_env", "get_algorithm_class", "MultiAgentEnv", "make_multi_agent", "PolicySpec",
           "Policy", "TorchPolicy", "TFPolicy", "RolloutWorker", "BaseEnv", "VectorEnv", "ExternalEnv"]
