"""RLlib equivalent (reference: ``rllib/``): PPO / DQN (IMPALA / APPO in ``algorithms.impala``),
vectorised env runners, GPU learners over RCCL, HIP GAE."""
from .algorithms import DQN, PPO, Algorithm, AlgorithmConfig, DQNConfig, PPOConfig, get_algorithm_class
from .env import register_env
from .policy.sample_batch import MultiAgentBatch, SampleBatch

__all__ = ["PPO", "PPOConfig", "DQN", "DQNConfig", "Algorithm", "AlgorithmConfig", "SampleBatch", "MultiAgentBatch",
           "register_env", "get_algorithm_class"]
