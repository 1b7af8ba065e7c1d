"""Blocks (reference: ``python/ray/data/block.py``, ``_internal/{arrow,pandas}_block.py``).

A block is either a ``pyarrow.Table`` (tabular sources) or a ``dict[str, np.ndarray]`` "numpy
block" (tensor-friendly: image batches stay ndarrays, zero conversion for
``batch_format="numpy"``). ``BlockAccessor`` hides the difference.
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Union

import numpy as np

try:
    import pyarrow as pa
except ImportError:  # pragma: no cover
    pa = None

Block = Union["pa.Table", Dict[str, np.ndarray]]


def _is_arrow(b):
    return pa is not None and isinstance(b, pa.Table)


def _is_pandas(b):
    try:
        import pandas as pd

        return isinstance(b, pd.DataFrame)
    except ImportError:
        return False


def _is_tensor_type(t) -> bool:
    from .extensions.tensor_extension import is_tensor_type

    return is_tensor_type(t)


def _tensor_to_numpy(col) -> np.ndarray:
    from .extensions.tensor_extension import tensor_column_to_numpy

    return tensor_column_to_numpy(col)


def _np_col(v):
    if isinstance(v, np.ndarray):
        return v
    if type(v).__name__ == "TensorArray":
        return v.to_numpy()
    if isinstance(v, list):
        try:
            arr = np.asarray(v)
            if arr.dtype == object and len(v) and isinstance(v[0], np.ndarray):
                return np.stack(v)
            return arr
        except (ValueError, TypeError):
            a = np.empty(len(v), dtype=object)
            a[:] = v
            return a
    try:
        import torch

        if isinstance(v, torch.Tensor):
            return v.detach().cpu().numpy()
    except ImportError:
        pass
    return np.asarray(v)


class BlockAccessor:
    def __init__(self, block):
        self.b = block

    @staticmethod
    def for_block(block) -> "BlockAccessor":
        return BlockAccessor(normalize_block(block))

    def num_rows(self) -> int:
        b = self.b
        if _is_arrow(b):
            return b.num_rows
        if not b:
            return 0
        return len(next(iter(b.values())))

    def size_bytes(self) -> int:
        b = self.b
        if _is_arrow(b):
            return b.nbytes
        return int(sum(getattr(v, "nbytes", 0) for v in b.values()))

    def column_names(self) -> List[str]:
        return list(self.b.column_names) if _is_arrow(self.b) else list(self.b.keys())

    def schema(self):
        b = self.b
        if _is_arrow(b):
            return b.schema
        return {k: (v.dtype, v.shape[1:]) for k, v in b.items()}

    def slice(self, start, end) -> Block:
        b = self.b
        if _is_arrow(b):
            return b.slice(start, end - start)
        return {k: v[start:end] for k, v in b.items()}

    def take(self, idx) -> Block:
        b = self.b
        if _is_arrow(b):
            return b.take(pa.array(np.asarray(idx, dtype=np.int64)))
        return {k: v[idx] for k, v in b.items()}

    def to_numpy(self) -> Dict[str, np.ndarray]:
        b = self.b
        if _is_arrow(b):
            out = {}
            for name in b.column_names:
                col = b.column(name)
                if _is_tensor_type(col.type):  # fixed-shape tensor column: one reshape
                    out[name] = _tensor_to_numpy(col)
                    continue
                try:
                    out[name] = col.to_numpy(zero_copy_only=False)
                except Exception:
                    out[name] = np.asarray(col.to_pylist(), dtype=object)
                if out[name].dtype == object and len(out[name]) and isinstance(out[name][0], (list, np.ndarray)):
                    try:
                        out[name] = np.stack([np.asarray(x) for x in out[name]])
                    except ValueError:
                        pass
            return out
        return dict(b)

    def to_pandas(self):
        import pandas as pd

        b = self.b
        if _is_arrow(b):
            return b.to_pandas()
        from .extensions import TensorArray

        cols = {}
        for k, v in b.items():
            cols[k] = TensorArray(v) if v.ndim > 1 else v
        return pd.DataFrame(cols)

    def to_arrow(self):
        b = self.b
        if _is_arrow(b):
            return b
        from .extensions.tensor_extension import to_tensor_block_column

        # ndim > 1 columns become ArrowTensorType columns: the row shape survives Arrow / Parquet
        return pa.table({k: to_tensor_block_column(v) for k, v in b.items()})

    def to_batch(self, fmt: str):
        if fmt in ("numpy", "default", None):
            return self.to_numpy()
        if fmt == "pandas":
            return self.to_pandas()
        if fmt in ("pyarrow", "arrow"):
            return self.to_arrow()
        raise ValueError(f"unknown batch_format {fmt}")

    def iter_rows(self) -> Iterator[Dict[str, Any]]:
        cols = self.to_numpy()
        n = self.num_rows()
        keys = list(cols)
        for i in range(n):
            yield {k: _py(cols[k][i]) for k in keys}

    # ------------------------------------------------------------------ reference API surface
    # (python/ray/data/block.py BlockAccessor; sorting / aggregation helpers live in the exchange
    # code of _internal/execution.py and work on these same blocks)
    def to_batch_format(self, batch_format: Optional[str]):
        return self.to_batch(batch_format)

    def to_default(self) -> Block:
        return self.b

    def to_block(self) -> Block:
        return self.b

    @staticmethod
    def batch_to_block(batch) -> Block:
        return normalize_block(batch)

    @staticmethod
    def builder():
        """A block builder: ``add(row)`` / ``add_block(block)`` then ``build()``."""
        return _BlockBuilder()

    def select(self, columns: List[str]) -> Block:
        if _is_arrow(self.b):
            return self.b.select(columns)
        return {c: self.b[c] for c in columns}

    def get_metadata(self, input_files=None, exec_stats=None) -> Dict[str, Any]:
        return {"num_rows": self.num_rows(), "size_bytes": self.size_bytes(), "schema": self.schema(),
                "input_files": list(input_files or []), "exec_stats": exec_stats}

    def random_shuffle(self, random_seed: Optional[int] = None) -> Block:
        perm = np.random.default_rng(random_seed).permutation(self.num_rows())
        return self.take(perm)

    def sample(self, n_samples: int, sort_key=None) -> Block:
        """``n_samples`` random rows (of the ``sort_key`` columns when given)."""
        n = self.num_rows()
        idx = np.random.default_rng().choice(n, size=min(int(n_samples), n), replace=False) if n else np.arange(0)
        out = BlockAccessor(self.take(np.sort(idx)))
        if sort_key is not None:
            cols = [sort_key] if isinstance(sort_key, str) else list(getattr(sort_key, "get_columns", lambda: sort_key)())
            return out.select(cols)
        return out.b

    def zip(self, other: Block) -> Block:
        """Columns of both blocks side by side (equal row counts; clashing names get a suffix)."""
        a, o = self.to_numpy(), BlockAccessor.for_block(other).to_numpy()
        if self.num_rows() != BlockAccessor.for_block(other).num_rows():
            raise ValueError("cannot zip blocks of different row counts")
        out = dict(a)
        for k, v in o.items():
            out[k if k not in out else f"{k}_1"] = v
        return out

    def sort_and_partition(self, boundaries: List[Any], sort_key) -> List[Block]:
        """Sort by ``sort_key`` (a column name) and cut at the boundary values."""
        key = sort_key if isinstance(sort_key, str) else list(getattr(sort_key, "get_columns", lambda: [sort_key])())[0]
        cols = self.to_numpy()
        order = np.argsort(cols[key], kind="stable")
        srt = {k: v[order] for k, v in cols.items()}
        cuts = np.searchsorted(srt[key], np.asarray(boundaries), side="left") if len(boundaries) else []
        bounds = [0] + list(cuts) + [len(order)]
        return [{k: v[a:b] for k, v in srt.items()} for a, b in zip(bounds[:-1], bounds[1:])]

    @staticmethod
    def merge_sorted_blocks(blocks: List[Block], sort_key) -> Block:
        key = sort_key if isinstance(sort_key, str) else list(getattr(sort_key, "get_columns", lambda: [sort_key])())[0]
        merged = BlockAccessor.for_block(concat_blocks(list(blocks))).to_numpy()
        if not merged:
            return {}
        order = np.argsort(merged[key], kind="stable")
        return {k: v[order] for k, v in merged.items()}

    def combine(self, key, aggs) -> Block:
        """Group this block by ``key`` and apply ``aggs`` (``AggregateFn`` objects from
        ``ray.data.aggregate``) into one row per group: the partial-aggregation step."""
        from .grouped_data import _aggregate_block

        return _aggregate_block(self.b, key, aggs)

    @staticmethod
    def aggregate_combined_blocks(blocks: List[Block], key, aggs) -> Block:
        from .grouped_data import _aggregate_block

        return _aggregate_block(concat_blocks(list(blocks)), key, aggs)


class _BlockBuilder:
    def __init__(self):
        self._rows: List[Dict] = []
        self._blocks: List[Block] = []

    def add(self, row: Dict) -> None:
        self._rows.append(dict(row))

    def add_block(self, block: Block) -> None:
        self._blocks.append(normalize_block(block))

    def num_rows(self) -> int:
        return len(self._rows) + sum(BlockAccessor(b).num_rows() for b in self._blocks)

    def build(self) -> Block:
        parts = list(self._blocks) + ([rows_to_block(self._rows)] if self._rows else [])
        return concat_blocks(parts) if parts else {}


def _py(x):
    if isinstance(x, np.generic):
        return x.item()
    return x


def normalize_block(x) -> Block:
    """Convert a UDF output / batch into a block."""
    if x is None:
        return {}
    if _is_arrow(x):
        return x
    if _is_pandas(x):
        if pa is not None:
            try:
                return pa.Table.from_pandas(x, preserve_index=False)
            except Exception:
                pass
        return {c: _np_col(x[c].array if type(x[c].array).__name__ == "TensorArray" else list(x[c]))
                for c in x.columns}
    if isinstance(x, dict):
        return {str(k): _np_col(v) for k, v in x.items()}
    if isinstance(x, list):
        return rows_to_block(x)
    raise TypeError(f"cannot convert {type(x)} to a block; return a dict of arrays, pandas or pyarrow")


def rows_to_block(rows: List[Any]) -> Block:
    if not rows:
        return {}
    if not isinstance(rows[0], dict):
        rows = [{"item": r} for r in rows]
    keys = list(rows[0].keys())
    return {k: _np_col([r[k] for r in rows]) for k in keys}


def concat_blocks(blocks: List[Block]) -> Block:
    blocks = [b for b in blocks if BlockAccessor(b).num_rows() > 0]
    if not blocks:
        return {}
    if len(blocks) == 1:
        return blocks[0]
    if all(_is_arrow(b) for b in blocks):
        return pa.concat_tables(blocks, promote_options="default")
    nps = [BlockAccessor(b).to_numpy() for b in blocks]
    keys = list(nps[0].keys())
    out = {}
    for k in keys:
        parts = [n[k] for n in nps]
        try:
            out[k] = np.concatenate(parts, axis=0)
        except ValueError:
            a = np.empty(sum(len(p) for p in parts), dtype=object)
            a[:] = [x for p in parts for x in p]
            out[k] = a
    return out


class BlockMetadata(dict):
    pass
