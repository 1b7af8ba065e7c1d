"""Dataset creation (reference: ``python/ray/data/read_api.py`` + ``datasource/*``)."""
from __future__ import annotations

import glob
import math
import os
from typing import Any, Dict, List, Optional, Union

import numpy as np

from .block import rows_to_block
from .dataset import Dataset, _cpus


def _default_parallelism(n_items: int, override: Optional[int]) -> int:
    if override and override > 0:
        return override
    return max(1, min(n_items, 2 * _cpus() if n_items > 0 else 1, 200))


def range(n: int, *, parallelism: int = -1, override_num_blocks: Optional[int] = None) -> Dataset:  # noqa: A001
    k = _default_parallelism(n, override_num_blocks or (parallelism if parallelism > 0 else None))
    inputs = []
    for i in builtins_range(k):
        lo = n * i // k
        hi = n * (i + 1) // k
        inputs.append(("read", _RangeRead(lo, hi)))
    return Dataset(inputs)


def range_tensor(n: int, *, shape=(1,), parallelism: int = -1, override_num_blocks=None) -> Dataset:
    k = _default_parallelism(n, override_num_blocks or (parallelism if parallelism > 0 else None))
    return Dataset([("read", _RangeRead(n * i // k, n * (i + 1) // k, tuple(shape))) for i in builtins_range(k)])


import builtins  # noqa: E402

builtins_range = builtins.range


class _RangeRead:
    def __init__(self, lo, hi, shape=None):
        self.lo, self.hi, self.shape = lo, hi, shape

    def __call__(self):
        ids = np.arange(self.lo, self.hi, dtype=np.int64)
        if self.shape is None:
            return {"id": ids}
        return {"data": np.broadcast_to(ids.reshape((-1,) + (1,) * len(self.shape)),
                                        (len(ids),) + self.shape).copy()}


def _put_blocks(blocks):
    from .._private.worker import _core, put

    from ._internal.execution import _meta

    core = _core()
    out = []
    for b in blocks:
        out.append(("ref", put(b), put(_meta(b))))
    return out


def from_items(items: List[Any], *, parallelism: int = -1, override_num_blocks=None) -> Dataset:
    from .._private.worker import _core

    _core()
    n = len(items)
    k = _default_parallelism(n, override_num_blocks or (parallelism if parallelism > 0 else None))
    k = max(1, min(k, n)) if n else 1
    blocks = [rows_to_block(items[n * i // k: n * (i + 1) // k]) for i in builtins_range(k)]
    return Dataset(_put_blocks(blocks))


def from_numpy(ndarrays) -> Dataset:
    from .._private.worker import _core

    _core()
    if isinstance(ndarrays, np.ndarray):
        ndarrays = [ndarrays]
    return Dataset(_put_blocks([{"data": a} for a in ndarrays]))


def from_numpy_refs(refs) -> Dataset:
    from .._private.worker import get

    return from_numpy(get(list(refs)))


def from_pandas(dfs) -> Dataset:
    from .._private.worker import _core

    from .block import normalize_block

    _core()
    if not isinstance(dfs, list):
        dfs = [dfs]
    return Dataset(_put_blocks([normalize_block(d) for d in dfs]))


def from_arrow(tables) -> Dataset:
    from .._private.worker import _core

    _core()
    if not isinstance(tables, list):
        tables = [tables]
    return Dataset(_put_blocks(tables))


def from_torch(dataset) -> Dataset:
    items = [dataset[i] for i in builtins_range(len(dataset))]
    return from_items([{"item": x} for x in items])


def from_huggingface(dataset) -> Dataset:
    return from_arrow(dataset.data.table if hasattr(dataset, "data") else dataset.with_format("arrow")[:])


def _expand_paths(paths, exts=None):
    if isinstance(paths, str):
        paths = [paths]
    out = []
    for p in paths:
        if os.path.isdir(p):
            for root, _, files in os.walk(p):
                for f in sorted(files):
                    if f.startswith(".") or f.startswith("_"):
                        continue
                    if exts is None or any(f.endswith(e) for e in exts):
                        out.append(os.path.join(root, f))
        elif any(c in p for c in "*?["):
            out.extend(sorted(glob.glob(p)))
        else:
            out.append(p)
    return sorted(out)


class _FileRead:
    def __init__(self, path, fmt, kwargs, include_paths=False):
        self.path, self.fmt, self.kwargs, self.include_paths = path, fmt, kwargs, include_paths

    def __call__(self):
        p, fmt, kw = self.path, self.fmt, self.kwargs
        if fmt == "parquet":
            import pyarrow.parquet as pq

            t = pq.read_table(p, columns=kw.get("columns"))
        elif fmt == "csv":
            import pyarrow.csv as pcsv

            t = pcsv.read_csv(p)
        elif fmt == "json":
            import pyarrow.json as pj

            t = pj.read_json(p)
        elif fmt == "text":
            with open(p, "r", encoding=kw.get("encoding", "utf-8")) as f:
                lines = f.read().splitlines()
            if kw.get("drop_empty_lines", True):
                lines = [l for l in lines if l.strip()]
            b = {"text": np.asarray(lines, dtype=object)}
            if self.include_paths:
                b["path"] = np.asarray([p] * len(lines), dtype=object)
            return b
        elif fmt == "numpy":
            return {"data": np.load(p, allow_pickle=False)}
        elif fmt == "binary":
            with open(p, "rb") as f:
                data = f.read()
            a = np.empty(1, dtype=object)
            a[0] = data
            b = {"bytes": a}
            if self.include_paths:
                b["path"] = np.asarray([p], dtype=object)
            return b
        elif fmt == "images":
            from PIL import Image  # optional dependency

            img = np.asarray(Image.open(p).convert(kw.get("mode", "RGB")))
            if kw.get("size"):
                img = np.asarray(Image.fromarray(img).resize(kw["size"][::-1]))
            b = {"image": img[None]}
            if self.include_paths:
                b["path"] = np.asarray([p], dtype=object)
            return b
        else:
            raise ValueError(fmt)
        if self.include_paths:
            import pyarrow as pa

            t = t.append_column("path", pa.array([p] * t.num_rows))
        return t


def _read(paths, fmt, exts, include_paths=False, **kw) -> Dataset:
    files = _expand_paths(paths, exts)
    if not files:
        raise ValueError(f"No input files found to read from paths {paths}")
    return Dataset([("read", _FileRead(f, fmt, kw, include_paths)) for f in files])


def read_parquet(paths, *, columns=None, include_paths=False, **kw) -> Dataset:
    return _read(paths, "parquet", [".parquet"], include_paths, columns=columns)


def read_csv(paths, *, include_paths=False, **kw) -> Dataset:
    return _read(paths, "csv", [".csv"], include_paths)


def read_json(paths, *, include_paths=False, **kw) -> Dataset:
    return _read(paths, "json", [".json", ".jsonl"], include_paths)


def read_text(paths, *, encoding="utf-8", drop_empty_lines=True, include_paths=False, **kw) -> Dataset:
    return _read(paths, "text", None, include_paths, encoding=encoding, drop_empty_lines=drop_empty_lines)


def read_numpy(paths, **kw) -> Dataset:
    return _read(paths, "numpy", [".npy"])


def read_binary_files(paths, *, include_paths=False, **kw) -> Dataset:
    return _read(paths, "binary", None, include_paths)


def read_images(paths, *, size=None, mode="RGB", include_paths=False, **kw) -> Dataset:
    return _read(paths, "images", [".png", ".jpg", ".jpeg", ".bmp", ".gif", ".tif", ".tiff"], include_paths,
                 size=size, mode=mode)


def read_datasource(datasource, *, parallelism: int = -1, **read_args) -> Dataset:
    tasks = datasource.get_read_tasks(parallelism if parallelism > 0 else 2 * _cpus(), **read_args)
    return Dataset([("read", t) for t in tasks])


class Datasource:
    """Custom datasource: implement ``get_read_tasks(parallelism) -> list of zero-arg callables``."""

    def get_read_tasks(self, parallelism: int, **kw):
        raise NotImplementedError
