"""``PolicySpec`` (reference: ``rllib/policy/policy.py``): how to build one policy of a
multi-agent setup. Spaces left as ``None`` are taken from the env agents mapped to the policy."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class PolicySpec:
    policy_class: Any = None
    observation_space: Any = None
    action_space: Any = None
    config: Optional[Dict] = field(default=None)
