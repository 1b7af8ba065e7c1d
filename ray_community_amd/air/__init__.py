from .config import CheckpointConfig, DatasetConfig, FailureConfig, RunConfig, ScalingConfig
from .result import Result

from typing import Dict, Union

import numpy as np

DataBatchType = Union["np.ndarray", "pandas.DataFrame", "pyarrow.Table", Dict[str, "np.ndarray"]]


class ResourceRequest:
    """Resources of one placement request as bundles (reference ``air/execution/resources/request.py``)."""

    def __init__(self, bundles, strategy: str = "PACK", *args, **kwargs):
        self.bundles = [dict(b) for b in bundles]
        self.strategy = strategy

    @property
    def head_bundle_is_empty(self):
        return not any(self.bundles[0].values())

    @property
    def required_resources(self):
        out = {}
        for b in self.bundles:
            for k, v in b.items():
                out[k] = out.get(k, 0.0) + v
        return out

    def __eq__(self, other):
        return isinstance(other, ResourceRequest) and (self.bundles, self.strategy) == (other.bundles, other.strategy)

    def __hash__(self):
        return hash((tuple(tuple(sorted(b.items())) for b in self.bundles), self.strategy))


class AcquiredResources:
    """Resources granted for a ResourceRequest: ``annotate_remote_entities`` pins actors/tasks
    to the request's placement group bundles."""

    def __init__(self, resource_request: ResourceRequest, placement_group=None):
        self.resource_request = resource_request
        self.placement_group = placement_group

    def annotate_remote_entities(self, entities):
        from ..util.scheduling_strategies import PlacementGroupSchedulingStrategy

        if self.placement_group is None:
            return list(entities)
        return [e.options(scheduling_strategy=PlacementGroupSchedulingStrategy(self.placement_group, i))
                for i, e in enumerate(entities)]


__all__ = ["DataBatchType", "ResourceRequest", "AcquiredResources", "ScalingConfig", "RunConfig", "CheckpointConfig", "FailureConfig", "DatasetConfig", "Result"]
