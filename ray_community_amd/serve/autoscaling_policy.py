"""Serve's default autoscaling policy (reference: python/ray/serve/autoscaling_policy.py), the
rule the controller applies each control-loop tick (serve/_private/controller.py ``_autoscale``):
replicas = ceil(total ongoing requests / target per replica), clamped to [min, max], with
``upscale_delay_s`` / ``downscale_delay_s`` hysteresis applied by the controller."""
from __future__ import annotations

import math
from typing import Any, Dict


def _get(cfg, key, default):
    return cfg.get(key, default) if isinstance(cfg, dict) else getattr(cfg, key, default)


def calculate_desired_num_replicas(autoscaling_config: Any, total_num_requests: float,
                                   num_running_replicas: int, **kw) -> int:
    target = _get(autoscaling_config, "target_ongoing_requests", None) or \
        _get(autoscaling_config, "target_num_ongoing_requests_per_replica", 1.0)
    lo = int(_get(autoscaling_config, "min_replicas", 1))
    hi = int(_get(autoscaling_config, "max_replicas", max(lo, 1)))
    if total_num_requests <= 0:
        return max(lo, 0)
    desired = math.ceil(float(total_num_requests) / max(float(target), 1e-9))
    return max(lo, min(hi, desired))


def default_autoscaling_policy(ctx: Dict, **kw) -> int:
    return calculate_desired_num_replicas(ctx["config"], ctx["total_num_requests"], ctx["current_num_replicas"])


__all__ = ["calculate_desired_num_replicas", "default_autoscaling_policy"]
