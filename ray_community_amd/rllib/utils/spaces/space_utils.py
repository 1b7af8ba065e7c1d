"""Helpers over (nested) action / observation spaces and the values they hold (reference:
``rllib/utils/spaces/space_utils.py``). Nested structures are dicts / tuples / lists of leaves
(dicts visited in sorted key order, as flattening does in the reference); no ``dm-tree``.
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional, Union

import numpy as np

from . import Box, Dict, Discrete, Space, Tuple


# ---------------------------------------------------------------------------------------- structs
def _is_node(x) -> bool:
    return isinstance(x, (dict, tuple, list))


def _flatten(x) -> list:
    if isinstance(x, dict):
        return [leaf for k in sorted(x) for leaf in _flatten(x[k])]
    if isinstance(x, (tuple, list)):
        return [leaf for v in x for leaf in _flatten(v)]
    return [x]


def _unflatten_as(like, leaves: list):
    it = iter(leaves)

    def build(node):
        if isinstance(node, dict):
            built = {k: build(node[k]) for k in sorted(node)}
            return {k: built[k] for k in node}
        if isinstance(node, (tuple, list)):
            return type(node)(build(v) for v in node)
        return next(it)

    return build(like)


def _map(fn: Callable, *structs):
    first = structs[0]
    if isinstance(first, dict):
        return {k: _map(fn, *(s[k] for s in structs)) for k in first}
    if isinstance(first, (tuple, list)):
        return type(first)(_map(fn, *vals) for vals in zip(*structs))
    return fn(*structs)


# ---------------------------------------------------------------------------------------- spaces
def get_original_space(space: Space) -> Space:
    """The space a preprocessor / wrapper flattened (``space.original_space`` chains), or ``space``."""
    while hasattr(space, "original_space"):
        space = space.original_space
    return space


def flatten_space(space: Space) -> List[Space]:
    """The primitive (non-Tuple / non-Dict) spaces of a nested space, in flattening order."""
    if isinstance(space, Tuple):
        return [p for s in space.spaces for p in flatten_space(s)]
    if isinstance(space, Dict):
        return [p for k in sorted(space.spaces) for p in flatten_space(space.spaces[k])]
    return [space]


def get_base_struct_from_space(space):
    """A Tuple / Dict space as the same-shaped python tuple / dict of its primitive spaces."""
    if isinstance(space, Tuple):
        return tuple(get_base_struct_from_space(s) for s in space.spaces)
    if isinstance(space, Dict):
        return {k: get_base_struct_from_space(s) for k, s in space.spaces.items()}
    return space


def get_dummy_batch_for_space(space: Space, batch_size: int = 32, *, fill_value: Union[float, int, str] = 0.0,
                              time_size: Optional[int] = None, time_major: bool = False,
                              one_hot_discrete: bool = False):
    """A batch of ``fill_value`` (or ``"random"`` samples) shaped for ``space``: leading dims
    ``[batch_size]`` or ``[batch_size, time_size]`` (``[time_size, batch_size]`` if time-major);
    ``batch_size=0`` means no batch dim. Discrete values can be one-hot encoded."""
    struct = get_base_struct_from_space(space)
    lead = [] if batch_size == 0 else [batch_size]
    if time_size is not None:
        lead = [time_size] + lead if time_major else lead + [time_size]

    def one(s):
        if isinstance(s, Discrete) and one_hot_discrete:
            shape, dtype = [s.n], np.float32
        else:
            shape, dtype = list(s.shape or ()), (s.dtype or np.float32)
        if fill_value == "random":
            n = int(np.prod(lead)) if lead else 1
            vals = np.stack([np.asarray(s.sample()) for _ in range(n)]) if n else np.zeros([0] + list(s.shape or ()))
            if isinstance(s, Discrete) and one_hot_discrete:
                vals = np.eye(s.n, dtype=np.float32)[vals.astype(np.int64)]
            return vals.reshape(lead + shape).astype(dtype)
        return np.full(lead + shape, fill_value, dtype=dtype)

    return _map(one, struct)


# ---------------------------------------------------------------------------------------- values
class BatchedNdArray(np.ndarray):
    """Marks an array that already has a batch dim (``batch(..., "auto")`` concatenates these)."""



def flatten_to_single_ndarray(input_):
    """A (nested) struct of arrays / scalars as ONE flat 1-D array (leaves raveled and
    concatenated); a plain array is returned unchanged."""
    if isinstance(input_, (list, tuple, dict)):
        return np.concatenate([np.reshape(np.asarray(x), [-1]) for x in _flatten(input_)], axis=0).flatten()
    return input_


def batch(list_of_structs: List[Any], *, individual_items_already_have_batch_dim: Union[bool, str] = False):
    """List of same-shaped structs -> struct of batches (stacked on a new axis 0, or concatenated
    when every item already carries a batch dim; ``"auto"``: concatenated if the leaves are
    ``BatchedNdArray`` views)."""
    if not list_of_structs:
        raise ValueError("Input `list_of_structs` does not contain any items.")
    concat = individual_items_already_have_batch_dim
    if concat == "auto":  # items marked as already batched (BatchedNdArray leaves) are concatenated
        concat = isinstance(_flatten(list_of_structs[0])[0], BatchedNdArray)
    fn = np.concatenate if concat else np.stack
    return _map(lambda *xs: fn([np.asarray(x) for x in xs], axis=0), *list_of_structs)


def unbatch(batches_struct) -> list:
    """Struct of batches -> list of per-item structs (the inverse of ``batch``)."""
    leaves = _flatten(batches_struct)
    n = len(leaves[0])
    return [_unflatten_as(batches_struct, [leaf[i] for leaf in leaves]) for i in range(n)]


def clip_action(action, action_space):
    """Box components clipped to their bounds (``action_space`` is a space or its base struct)."""
    struct = get_base_struct_from_space(action_space) if isinstance(action_space, Space) else action_space
    return _map(lambda a, s: np.clip(a, s.low, s.high) if isinstance(s, Box) else a, action, struct)


def _bounded(s) -> bool:
    return isinstance(s, Box) and np.all(np.isfinite(s.low)) and np.all(np.isfinite(s.high))


def unsquash_action(action, action_space_struct):
    """[-1, 1] policy outputs -> the bounded float Box ranges (clipped); integer Boxes are shifted
    by ``low`` (the reference's convention); other components pass through."""
    struct = get_base_struct_from_space(action_space_struct) if isinstance(action_space_struct, Space) \
        else action_space_struct

    def one(a, s):
        if _bounded(s) and np.issubdtype(s.dtype, np.floating):
            return np.clip(s.low + (np.asarray(a) + 1.0) * (s.high - s.low) / 2.0, s.low, s.high)
        if isinstance(s, Box) and np.issubdtype(s.dtype, np.integer):
            return np.asarray(a) + s.low
        return a

    return _map(one, action, struct)


def normalize_action(action, action_space_struct):
    """The inverse of ``unsquash_action``: bounded float Box values -> [-1, 1]."""
    struct = get_base_struct_from_space(action_space_struct) if isinstance(action_space_struct, Space) \
        else action_space_struct

    def one(a, s):
        if _bounded(s) and np.issubdtype(s.dtype, np.floating):
            return (np.asarray(a) - s.low) * 2.0 / (s.high - s.low) - 1.0
        if isinstance(s, Box) and np.issubdtype(s.dtype, np.integer):
            return np.asarray(a) - s.low
        return a

    return _map(one, action, struct)


def convert_element_to_space_type(element: Any, sampled_element: Any) -> Any:
    """``element`` cast leaf by leaf to the dtypes / python types of ``sampled_element`` (a sample
    of the space), so e.g. float64 observations pass a float32 Box's ``contains``."""

    def one(e, s):
        if isinstance(s, np.ndarray):
            return np.asarray(e, dtype=s.dtype)
        if isinstance(s, (np.integer, int)) and not isinstance(s, bool):
            return int(e)
        if isinstance(s, (np.floating, float)):
            return float(e)
        return e

    return _map(one, element, sampled_element)


__all__ = ["BatchedNdArray", "get_original_space", "flatten_space", "get_base_struct_from_space", "get_dummy_batch_for_space",
           "flatten_to_single_ndarray", "batch", "unbatch", "clip_action", "unsquash_action", "normalize_action",
           "convert_element_to_space_type"]
