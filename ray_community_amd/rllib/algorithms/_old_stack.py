"""Old-API-stack policy class names the reference algorithm packages export
(``PPOTorchPolicy``, ``DQNTorchPolicy``, ``SACTorchPolicy``, the TF variants, RNNSAC).

Training runs on RLModules + Learners here; the torch names resolve to ``TorchPolicy``
subclasses over the algorithm's RLModule (action computation and weights, the parts of the
old Policy API that do not depend on the old training loop). The TensorFlow names raise
ImportError (TensorFlow is not installed)."""
from __future__ import annotations

from ..policy.policy import TorchPolicy

_TORCH = {"PPOTorchPolicy": "PPO", "DQNTorchPolicy": "DQN", "SACTorchPolicy": "SAC"}
_TF = {"PPOTF1Policy", "PPOTF2Policy", "DQNTFPolicy", "SACTFPolicy"}
_UNSUPPORTED = {"RNNSAC", "RNNSACConfig", "RNNSACTorchPolicy"}
_cache = {}


def policy_alias(name: str, module: str):
    if name in _TORCH:
        if name not in _cache:
            algo = _TORCH[name]

            def _init(self, observation_space, action_space, config=None, model=None):
                cfg = dict(config or {})
                if algo == "SAC":
                    cfg.setdefault("module_class", "sac")
                if algo == "DQN":
                    cfg.setdefault("q_head", True)
                TorchPolicy.__init__(self, observation_space, action_space, cfg, model)

            _cache[name] = type(name, (TorchPolicy,), {"__init__": _init, "__module__": module,
                                                       "__doc__": f"{algo}'s RLModule behind the old Policy API."})
        return _cache[name]
    if name in _TF or name in _UNSUPPORTED:  # importable names whose construction explains the gap
        msg = (f"{name}: TensorFlow is not installed; use the torch RLModule stack" if name in _TF else
               f"{name}: the recurrent SAC of the old API stack is not provided; use SAC, or PPO with "
               f"model={{'use_lstm': True}}")
        if name not in _cache:
            def _init(self, *a, **k):
                raise ImportError(msg)

            _cache[name] = type(name, (), {"__init__": _init, "__module__": module, "__doc__": msg})
        return _cache[name]
    raise AttributeError(f"module {module!r} has no attribute {name!r}")
