from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig
from .callbacks import DefaultCallbacks, RLlibCallback, make_multi_callbacks
from .cql import CQL, CQLConfig
from .dqn import DQN, DQNConfig
from .dreamerv3 import DreamerV3, DreamerV3Config
from .impala import APPO, IMPALA, APPOConfig, IMPALAConfig
from .marwil import BC, MARWIL, BCConfig, MARWILConfig
from .ppo import PPO, PPOConfig
from .sac import SAC, SACConfig
from .registry import ALGORITHMS, get_algorithm_class

Impala, ImpalaConfig = IMPALA, IMPALAConfig  # the reference exports both spellings

__all__ = ["Impala", "ImpalaConfig", "Algorithm", "AlgorithmConfig", "DefaultCallbacks", "RLlibCallback", "make_multi_callbacks", "PPO", "PPOConfig", "DQN", "DQNConfig", "DreamerV3", "DreamerV3Config", "IMPALA", "IMPALAConfig", "APPO", "APPOConfig", "SAC", "SACConfig", "CQL", "CQLConfig", "MARWIL", "MARWILConfig", "BC", "BCConfig", "get_algorithm_class", "ALGORITHMS"]
