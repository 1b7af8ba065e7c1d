"""Legacy ``ray.air.session`` shims (reference: ``python/ray/air/session.py``)."""
from ..train import get_checkpoint, get_context, get_dataset_shard, report


def get_world_rank():
    return get_context().get_world_rank()


def get_world_size():
    return get_context().get_world_size()


def get_local_rank():
    return get_context().get_local_rank()
