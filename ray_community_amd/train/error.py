"""``ray.train.error`` (reference: python/ray/train/error.py)."""


class SessionMisuseError(Exception):
    """A Train session function (report, get_checkpoint, ...) called outside a training worker."""
