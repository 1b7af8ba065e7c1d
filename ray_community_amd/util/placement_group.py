"""Placement groups (reference: ``python/ray/util/placement_group.py``)."""
from __future__ import annotations

from typing import Dict, List, Optional

from .._private.ids import PlacementGroupID, new_id

VALID_STRATEGIES = ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD")


class PlacementGroup:
    def __init__(self, id: PlacementGroupID, bundle_cache: Optional[List[Dict]] = None, strategy: str = "PACK"):
        self.id = id
        self.bundle_cache = bundle_cache
        self.strategy = strategy

    @staticmethod
    def empty():
        return PlacementGroup(PlacementGroupID.nil())

    def is_empty(self):
        return self.id.is_nil()

    def ready(self):
        """An ObjectRef that resolves when the group's bundles are reserved."""
        from .._private.worker import _core
        from ..remote_function import RemoteFunction

        pg = self

        def _ready():
            return True

        # a zero-resource task inside the group: it can only run once the group is placed
        f = RemoteFunction(_ready, {"num_cpus": 0, "max_retries": 0})
        from .scheduling_strategies import PlacementGroupSchedulingStrategy

        return f.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg, -1)).remote()

    def wait(self, timeout_seconds: float = 30) -> bool:
        from .._private.worker import _core

        return bool(_core().client.call("pg_ready", self.id.binary(), timeout_seconds))

    @property
    def bundle_specs(self) -> List[Dict]:
        if self.bundle_cache is None:
            from .._private.worker import _core

            t = _core().client.call("pg_table", self.id.binary())
            self.bundle_cache = [t["bundles"][i] for i in sorted(t["bundles"])] if t else []
        return self.bundle_cache

    @property
    def bundle_count(self):
        return len(self.bundle_specs)

    def __eq__(self, other):
        return isinstance(other, PlacementGroup) and other.id == self.id

    def __hash__(self):
        return hash(self.id)

    def __repr__(self):
        return f"PlacementGroup({self.id.hex()})"


def placement_group(bundles: List[Dict[str, float]], strategy: str = "PACK", name: str = "",
                    lifetime: Optional[str] = None, _max_cpu_fraction_per_node: float = 1.0,
                    _soft_target_node_id: Optional[str] = None) -> PlacementGroup:
    from .._private.worker import _core

    validate_placement_group(bundles, strategy, lifetime, _max_cpu_fraction_per_node, _soft_target_node_id)
    norm = [{k: float(v) for k, v in b.items()} for b in bundles]
    pid = PlacementGroupID(new_id())
    _core().client.call("create_pg", pid.binary(), norm, strategy, name, lifetime)
    return PlacementGroup(pid, norm, strategy)


def validate_placement_group(bundles: List[Dict[str, float]], strategy: str = "PACK", lifetime: Optional[str] = None,
                             _max_cpu_fraction_per_node: float = 1.0,
                             _soft_target_node_id: Optional[str] = None) -> bool:
    """Check ``placement_group`` arguments; raises ValueError on invalid ones, True otherwise."""
    if strategy not in VALID_STRATEGIES:
        raise ValueError(f"Invalid placement group strategy {strategy}. Supported strategies are: {VALID_STRATEGIES}.")
    if not bundles:
        raise ValueError("The placement group `bundles` argument cannot contain an empty list")
    for b in bundles:
        if not isinstance(b, dict) or not b:
            raise ValueError(f"Bundles must be non-empty dicts, got {b!r}")
        if all(v == 0 for v in b.values()):
            raise ValueError(f"Bundles cannot be an empty dictionary or resources with only 0 values. Bundles: {bundles}")
        for k, v in b.items():
            if v < 0:
                raise ValueError("resource quantities must be >= 0")
    if lifetime not in (None, "detached"):
        raise ValueError("placement group `lifetime` argument must be either `None` or 'detached'")
    if not 0 < _max_cpu_fraction_per_node <= 1:
        raise ValueError("_max_cpu_fraction_per_node must be in (0, 1]")
    if _soft_target_node_id is not None and strategy != "STRICT_PACK":
        raise ValueError("_soft_target_node_id only works with STRICT_PACK placement groups")
    return True


def remove_placement_group(placement_group: PlacementGroup):
    from .._private.worker import _core

    _core().client.call("remove_pg", placement_group.id.binary())


def get_placement_group(placement_group_name: str) -> PlacementGroup:
    from .._private.worker import _core

    info = _core().client.call("get_named_pg", placement_group_name)
    if info is None:
        raise ValueError(f"Failed to look up placement group with name: {placement_group_name}")
    return PlacementGroup(PlacementGroupID(info["pg_id"]), info["bundles"], info["strategy"])


def placement_group_table(placement_group: Optional[PlacementGroup] = None) -> dict:
    from .._private.worker import _core

    return _core().client.call("pg_table", placement_group.id.binary() if placement_group else None)


def get_current_placement_group() -> Optional[PlacementGroup]:
    from .._private.core_worker import _core

    if _core is None:
        return None
    pg_id = getattr(_core.ctx, "pg_id", None)
    if pg_id is None:
        return None
    return PlacementGroup(PlacementGroupID(pg_id))


def check_placement_group_index(placement_group, bundle_index):
    if placement_group is None:
        if bundle_index != -1:
            raise ValueError("If placement_group is not set, the value of bundle_index must be -1.")
    elif bundle_index >= placement_group.bundle_count or bundle_index < -1:
        raise ValueError(f"placement group bundle index {bundle_index} is invalid.")
