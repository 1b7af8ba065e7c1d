"""Tensor columns for Arrow tables and pandas DataFrames (reference: ``python/ray/data/extensions``
over ``air/util/tensor_extensions``: ``ArrowTensorType`` / ``ArrowTensorArray``, ``TensorDtype`` /
``TensorArray``).

A column whose every row is an ndarray of one fixed shape (an image batch, an embedding matrix)
is stored in Arrow as ``ArrowTensorType(shape, value_type)``: an extension type over a
``FixedSizeList<value_type>[prod(shape)]`` storage, so the values stay one contiguous buffer
(``from_numpy`` / ``to_numpy`` are one reshape, no per-row Python objects) and the shape survives
Arrow IPC, the object store and Parquet files (the type is registered with pyarrow, and its
shape is the extension metadata). In pandas the same column is a ``TensorArray`` of dtype
``TensorDtype(shape, dtype)``; conversions both ways go through the extension hooks
(``__arrow_array__`` / ``__from_arrow__``), so ``pa.Table.from_pandas`` and ``Table.to_pandas``
keep the tensors intact.
"""
from __future__ import annotations

import json
import numbers
from typing import Sequence, Tuple

import numpy as np
import pandas as pd
import pyarrow as pa
from pandas.api.extensions import ExtensionArray, ExtensionDtype, register_extension_dtype

_EXT_NAME = "ray_community_amd.data.tensor"


def _prod(shape) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n


class ArrowTensorType(pa.ExtensionType):
    """Fixed-shape tensor per row. ``shape`` excludes the row axis; ``dtype`` is the element
    Arrow type (or a numpy dtype)."""

    def __init__(self, shape: Sequence[int], dtype):
        self._shape = tuple(int(s) for s in shape)
        if not isinstance(dtype, pa.DataType):
            dtype = pa.from_numpy_dtype(np.dtype(dtype))
        super().__init__(pa.list_(dtype, max(1, _prod(self._shape))), _EXT_NAME)

    @property
    def shape(self) -> Tuple[int, ...]:
        return self._shape

    @property
    def scalar_type(self) -> pa.DataType:
        return self.storage_type.value_type

    def numpy_dtype(self) -> np.dtype:
        return np.dtype(self.scalar_type.to_pandas_dtype())

    def __arrow_ext_serialize__(self) -> bytes:
        return json.dumps({"shape": list(self._shape)}).encode()

    @classmethod
    def __arrow_ext_deserialize__(cls, storage_type, serialized):
        meta = json.loads(serialized.decode() or "{}")
        return cls(meta.get("shape", []), storage_type.value_type)

    def __arrow_ext_class__(self):
        return ArrowTensorArray

    def to_pandas_dtype(self):
        return TensorDtype(self._shape, self.numpy_dtype())

    def __reduce__(self):
        return ArrowTensorType, (self._shape, self.scalar_type)

    def __str__(self):
        return f"ArrowTensorType(shape={self._shape}, dtype={self.scalar_type})"

    __repr__ = __str__


class ArrowTensorArray(pa.ExtensionArray):
    """An Arrow array of fixed-shape tensors (one per row)."""

    @classmethod
    def from_numpy(cls, arr) -> "ArrowTensorArray":
        """``arr``: ``[rows, *shape]`` ndarray (or a sequence of equally shaped ndarrays)."""
        if isinstance(arr, (list, tuple)):
            arr = np.stack([np.asarray(a) for a in arr]) if len(arr) else np.empty((0,))
        if np.ndim(arr) == 0:
            raise ValueError("a tensor column needs a row axis")
        arr = np.ascontiguousarray(arr)
        shape = arr.shape[1:]
        values = pa.array(arr.reshape(-1))
        storage = pa.FixedSizeListArray.from_arrays(values, max(1, _prod(shape)))
        return pa.ExtensionArray.from_storage(ArrowTensorType(shape, values.type), storage)

    def to_numpy(self, zero_copy_only: bool = False) -> np.ndarray:
        t = self.type
        values = self.storage.flatten()  # honours the array's offset
        out = values.to_numpy(zero_copy_only=zero_copy_only)
        return out.reshape((len(self),) + t.shape)

    def to_pylist(self):
        return list(self.to_numpy())


def tensor_column_to_numpy(col) -> np.ndarray:
    """An ``ArrowTensorType`` column (Array or ChunkedArray) as one ``[rows, *shape]`` ndarray."""
    if isinstance(col, pa.ChunkedArray):
        chunks = [c.to_numpy() for c in col.chunks]
        if not chunks:
            t = col.type
            return np.empty((0,) + t.shape, dtype=t.numpy_dtype())
        return chunks[0] if len(chunks) == 1 else np.concatenate(chunks)
    return col.to_numpy()


def is_tensor_type(t) -> bool:
    return isinstance(t, ArrowTensorType)


# ---------------------------------------------------------------------------------------- pandas
@register_extension_dtype
class TensorDtype(ExtensionDtype):
    """pandas dtype of a ``TensorArray`` column: element shape + numpy element dtype."""

    _metadata = ("_shape", "_dtype")
    base = None

    def __init__(self, shape: Sequence[int] = (), dtype=np.float64):
        self._shape = tuple(int(s) for s in shape)
        self._dtype = np.dtype(dtype)

    @property
    def shape(self):
        return self._shape

    @property
    def element_dtype(self) -> np.dtype:
        return self._dtype

    @property
    def type(self):
        return np.ndarray

    @property
    def kind(self):
        return "O"

    @property
    def name(self) -> str:
        return f"TensorDtype(shape={self._shape}, dtype={self._dtype})"

    @classmethod
    def construct_array_type(cls):
        return TensorArray

    @classmethod
    def construct_from_string(cls, string):
        if not isinstance(string, str):
            raise TypeError(f"'construct_from_string' expects a string, got {type(string)}")
        if string.startswith("TensorDtype(shape=") and string.endswith(")"):
            body = string[len("TensorDtype(shape="):-1]
            shape_s, _, dt = body.rpartition(", dtype=")
            shape = tuple(int(x) for x in shape_s.strip("()").split(",") if x.strip())
            return cls(shape, np.dtype(dt))
        raise TypeError(f"Cannot construct a 'TensorDtype' from '{string}'")

    def __from_arrow__(self, array):
        return TensorArray(tensor_column_to_numpy(array))


class TensorArray(ExtensionArray):
    """A pandas column of equally shaped ndarrays, held as one ``[rows, *shape]`` ndarray.
    Row access returns the row's ndarray; slicing, masking and ``take`` return TensorArrays."""

    def __init__(self, values):
        if isinstance(values, TensorArray):
            values = values._v
        elif not isinstance(values, np.ndarray):
            values = np.stack([np.asarray(v) for v in values]) if len(values) else np.empty((0,))
        if values.ndim == 0:
            raise ValueError("TensorArray needs a row axis")
        self._v = values

    # -- construction
    @classmethod
    def _from_sequence(cls, scalars, *, dtype=None, copy=False):
        if isinstance(scalars, TensorArray):
            v = scalars._v
        else:
            v = np.stack([np.asarray(s) for s in scalars]) if len(scalars) else np.empty((0,))
        if dtype is not None and isinstance(dtype, TensorDtype):
            v = v.astype(dtype.element_dtype, copy=False)
        return cls(v.copy() if copy else v)

    @classmethod
    def _from_factorized(cls, values, original):
        raise NotImplementedError("TensorArray cannot be factorized (tensors are not hashable)")

    @classmethod
    def _concat_same_type(cls, to_concat):
        return cls(np.concatenate([t._v for t in to_concat]))

    # -- the array protocol pandas relies on
    @property
    def dtype(self) -> TensorDtype:
        return TensorDtype(self._v.shape[1:], self._v.dtype)

    @property
    def nbytes(self) -> int:
        return int(self._v.nbytes)

    @property
    def numpy_shape(self):
        return self._v.shape

    def __len__(self) -> int:
        return len(self._v)

    def __getitem__(self, item):
        if isinstance(item, numbers.Integral):
            return self._v[item]
        if isinstance(item, tuple) and len(item) and isinstance(item[0], numbers.Integral):
            return self._v[item]
        if isinstance(item, (pd.Series, pd.Index)):
            item = item.to_numpy()
        return TensorArray(self._v[item])

    def __setitem__(self, key, value):
        if isinstance(value, TensorArray):
            value = value._v
        self._v[key] = value

    def __iter__(self):
        return iter(self._v)

    def __array__(self, dtype=None, copy=None):
        out = np.empty(len(self._v), dtype=object)
        for i in range(len(self._v)):
            out[i] = self._v[i]
        return out

    def to_numpy(self, dtype=None, copy=False, na_value=None):
        """The ``[rows, *shape]`` ndarray."""
        v = self._v if dtype is None else self._v.astype(dtype)
        return v.copy() if copy else v

    def isna(self) -> np.ndarray:
        if self._v.dtype.kind == "f":
            return np.isnan(self._v.reshape(len(self._v), -1)).all(axis=1) if self._v.ndim > 1 else np.isnan(self._v)
        return np.zeros(len(self._v), dtype=bool)

    def take(self, indices, *, allow_fill=False, fill_value=None):
        idx = np.asarray(indices, dtype=np.int64)
        if allow_fill:
            missing = idx < 0
            if missing.any():
                out = self._v[np.where(missing, 0, idx)].copy()
                if fill_value is None or (isinstance(fill_value, float) and np.isnan(fill_value)):
                    if out.dtype.kind != "f":
                        out = out.astype(np.float64)
                    out[missing] = np.nan
                else:
                    out[missing] = fill_value
                return TensorArray(out)
        return TensorArray(self._v[idx])

    def copy(self):
        return TensorArray(self._v.copy())

    def __eq__(self, other):
        o = other._v if isinstance(other, TensorArray) else other
        return (self._v == o).reshape(len(self._v), -1).all(axis=1)

    # -- to Arrow
    def __arrow_array__(self, type=None):
        return ArrowTensorArray.from_numpy(self._v)

    def __repr__(self):
        return f"<TensorArray shape={self._v.shape} dtype={self._v.dtype}>"


try:  # one registration per process (re-imports under another module name must not fail)
    pa.register_extension_type(ArrowTensorType((0,), pa.int8()))
except pa.ArrowKeyError:
    pass


def to_tensor_block_column(v: np.ndarray):
    """The Arrow column for a numpy block column: an ``ArrowTensorArray`` for ndim > 1."""
    if v.ndim > 1:
        return ArrowTensorArray.from_numpy(v)
    return pa.array(v) if v.dtype != object else pa.array(list(v))


__all__ = ["ArrowTensorType", "ArrowTensorArray", "TensorDtype", "TensorArray", "tensor_column_to_numpy",
           "is_tensor_type", "to_tensor_block_column"]
