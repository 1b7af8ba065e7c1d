"""Serializer add-ons (reference: python/ray/util/serialization_addons.py): custom reducers for
types cloudpickle cannot handle on its own. Pydantic v2 models and Starlette requests pickle as
they are here; the registration helpers are kept so code calling them keeps working, and
``apply(serialization_context)`` runs every registration."""
from __future__ import annotations


def register_pydantic_serializer(serialization_context=None) -> None:
    """Pydantic v2 models pickle natively; nothing to register."""
    try:
        import pydantic  # noqa: F401
    except ImportError:
        return


def register_starlette_serializer(serialization_context=None) -> None:
    """Starlette ``Request`` objects carry a live receive channel and are never sent between
    processes here (Serve hands replicas a pickled request scope + body instead)."""
    try:
        import starlette.requests  # noqa: F401
    except ImportError:
        return


def apply(serialization_context=None) -> None:
    register_pydantic_serializer(serialization_context)
    register_starlette_serializer(serialization_context)
