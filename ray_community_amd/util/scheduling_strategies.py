"""Scheduling strategies (reference: ``python/ray/util/scheduling_strategies.py``)."""
from __future__ import annotations

from typing import Dict, Optional, Union


class PlacementGroupSchedulingStrategy:
    def __init__(self, placement_group, placement_group_bundle_index: int = -1,
                 placement_group_capture_child_tasks: Optional[bool] = None):
        self.placement_group = placement_group
        self.placement_group_bundle_index = placement_group_bundle_index
        self.placement_group_capture_child_tasks = placement_group_capture_child_tasks


class NodeAffinitySchedulingStrategy:
    def __init__(self, node_id: str, soft: bool, _spill_on_unavailable: bool = False, _fail_on_unavailable: bool = False):
        self.node_id = node_id
        self.soft = soft
        self._spill_on_unavailable = _spill_on_unavailable
        self._fail_on_unavailable = _fail_on_unavailable


class In:
    def __init__(self, *values):
        self.values = list(values)


class NotIn:
    def __init__(self, *values):
        self.values = list(values)


class Exists:
    pass


class DoesNotExist:
    pass


class NodeLabelSchedulingStrategy:
    def __init__(self, hard: Dict, *, soft: Optional[Dict] = None):
        self.hard = hard
        self.soft = soft


def normalize_label_selector(sel) -> list:
    """``label_selector`` / ``NodeLabelSchedulingStrategy(hard=...)`` as (key, op, values) clauses
    the head's scheduler understands. Values: ``"v"`` (equals), ``"!v"`` (not equals),
    ``"in(a,b)"`` / ``"!in(a,b)"``, or the ``In`` / ``NotIn`` / ``Exists`` / ``DoesNotExist``
    objects (reference: ``python/ray/util/scheduling_strategies.py``, label selectors)."""
    out = []
    for key, v in (sel or {}).items():
        if isinstance(v, In):
            out.append((key, "in", [str(x) for x in v.values]))
        elif isinstance(v, NotIn):
            out.append((key, "not_in", [str(x) for x in v.values]))
        elif isinstance(v, Exists) or v is Exists:
            out.append((key, "exists", []))
        elif isinstance(v, DoesNotExist) or v is DoesNotExist:
            out.append((key, "not_exists", []))
        elif isinstance(v, str):
            neg = v.startswith("!")
            body = v[1:] if neg else v
            if body.startswith("in(") and body.endswith(")"):
                vals = [x.strip() for x in body[3:-1].split(",") if x.strip()]
            else:
                vals = [body]
            out.append((key, "not_in" if neg else "in", vals))
        else:
            raise TypeError(f"label selector value for {key!r} must be a string or In/NotIn/Exists/DoesNotExist")
    return out


SchedulingStrategyT = Union[None, str, PlacementGroupSchedulingStrategy, NodeAffinitySchedulingStrategy,
                            NodeLabelSchedulingStrategy]
