"""Ray Train equivalent (reference: ``python/ray/train``)."""
from ._internal.session import TrainContext, get_session


def report(metrics, checkpoint=None):
    """Report metrics (and optionally a Checkpoint) from a training worker."""
    get_session().report(metrics, checkpoint=checkpoint)


def get_context() -> TrainContext:
    return get_session().context


def get_checkpoint():
    return get_session().checkpoint


def get_dataset_shard(name: str = "train"):
    return get_session().dataset_shards.get(name)
