"""RLlib equivalent (reference: ``rllib/``): PPO / DQN / IMPALA / APPO / SAC / CQL / MARWIL / BC,
vectorised env runners, GPU learners over RCCL, HIP GAE."""
from .algorithms import (APPO, BC, CQL, DQN, IMPALA, MARWIL, PPO, BCConfig, MARWILConfig, Algorithm, AlgorithmConfig, APPOConfig, DQNConfig, IMPALAConfig,
                         PPOConfig, SAC, SACConfig, CQLConfig, get_algorithm_class)
from .env import MultiAgentEnv, make_multi_agent, register_env
from .policy import PolicySpec
from .policy.sample_batch import MultiAgentBatch, SampleBatch

__all__ = ["PPO", "PPOConfig", "IMPALA", "IMPALAConfig", "APPO", "APPOConfig", "SAC", "SACConfig", "CQL", "CQLConfig", "MARWIL", "MARWILConfig", "BC", "BCConfig", "DQN", "DQNConfig", "Algorithm", "AlgorithmConfig", "SampleBatch", "MultiAgentBatch",
           "register_env", "get_algorithm_class", "MultiAgentEnv", "make_multi_agent", "PolicySpec"]
