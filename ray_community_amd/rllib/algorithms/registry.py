"""Algorithm registry (reference: ``rllib/algorithms/registry.py``)."""


def _ppo():
    from .ppo import PPO, PPOConfig

    return PPO, PPOConfig()


def _dqn():
    from .dqn import DQN, DQNConfig

    return DQN, DQNConfig()


def _impala():
    from .impala import IMPALA, IMPALAConfig

    return IMPALA, IMPALAConfig()


def _appo():
    from .impala import APPO, APPOConfig

    return APPO, APPOConfig()


def _sac():
    from .sac import SAC, SACConfig

    return SAC, SACConfig()


def _cql():
    from .cql import CQL, CQLConfig

    return CQL, CQLConfig()


def _marwil():
    from .marwil import MARWIL, MARWILConfig

    return MARWIL, MARWILConfig()


def _bc():
    from .marwil import BC, BCConfig

    return BC, BCConfig()


def _dreamerv3():
    from .dreamerv3 import DreamerV3, DreamerV3Config

    return DreamerV3, DreamerV3Config()


ALGORITHMS = {"PPO": _ppo, "DQN": _dqn, "IMPALA": _impala, "APPO": _appo, "SAC": _sac, "CQL": _cql, "MARWIL": _marwil,
              "BC": _bc, "DreamerV3": _dreamerv3}


def get_algorithm_class(name: str, return_config: bool = False):
    cls, cfg = ALGORITHMS[name]()
    return (cls, cfg) if return_config else cls
