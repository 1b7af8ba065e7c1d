"""Collective types (reference: ``python/ray/util/collective/types.py``)."""
from enum import Enum


class Backend(str, Enum):
    NCCL = "nccl"
    GLOO = "gloo"

    @classmethod
    def _missing_(cls, value):
        v = str(value).lower()
        if v in ("rccl", "nccl", "backend.nccl"):
            return cls.NCCL
        if v in ("gloo", "backend.gloo", "torch_gloo"):
            return cls.GLOO
        return None

    def __str__(self):
        return self.value


class ReduceOp(Enum):
    SUM = 0
    PRODUCT = 1
    MIN = 2
    MAX = 3
    AVG = 4
