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


def _expand_paths(paths, exts=None, bases=None):
    """Input files under ``paths``; ``bases`` (optional dict) receives file -> the directory it
    was found under (the root for hive partition discovery)."""
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
                        if bases is not None:
                            bases[out[-1]] = p
        elif any(c in p for c in "*?["):
            out.extend(sorted(glob.glob(p)))
        else:
            out.append(p)
    return sorted(out)


def _hive_fields(path, base):
    """``col=value`` directory components between ``base`` and the file (hive partitioning)."""
    if not base:
        return []
    rel = os.path.relpath(os.path.dirname(path), base)
    out = []
    for part in ([] if rel in (".", "") else rel.split(os.sep)):
        if "=" in part:
            k, v = part.split("=", 1)
            out.append((k, v))
    return out


class _FileRead:
    def __init__(self, path, fmt, kwargs, include_paths=False, base=None):
        self.path, self.fmt, self.kwargs, self.include_paths = path, fmt, kwargs, include_paths
        self.base = base

    def __call__(self):
        p, fmt, kw = self.path, self.fmt, self.kwargs
        if fmt == "parquet":
            import pyarrow.parquet as pq

            cols = kw.get("columns")
            if cols is not None and kw.get("partitioning", "hive") == "hive":
                have = set(pq.read_schema(p).names)  # partition columns live in the path, not the file
                cols = [c for c in cols if c in have]
            t = pq.read_table(p, columns=cols, filters=kw.get("filter"))
        elif fmt == "csv":
            import pyarrow.csv as pcsv

            t = pcsv.read_csv(p, **{k: kw[k] for k in ("read_options", "parse_options", "convert_options")
                                    if kw.get(k) is not None})
        elif fmt == "json":
            import pyarrow.json as pj

            t = pj.read_json(p, **{k: kw[k] for k in ("read_options", "parse_options") if kw.get(k) is not None})
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
        part = kw.get("partitioning", "hive")
        if part is not None:
            import pyarrow as pa

            cols = kw.get("columns")
            if part == "hive":
                fields = _hive_fields(p, self.base)
            else:  # a Partitioning object (HIVE or DIRECTORY; base_dir defaults to the read root)
                from .partitioning import Partitioning, PathPartitionParser

                if not part.base_dir and self.base:
                    part = Partitioning(part.style, self.base, part.field_names, part.field_types)
                fields = list(PathPartitionParser(part)(p).items())
            for k, v in fields:
                if k not in t.column_names and (cols is None or k in cols):
                    t = t.append_column(k, pa.array([v] * t.num_rows) if not isinstance(v, str)
                                        else pa.array([v] * t.num_rows, type=pa.string()))
            if cols is not None and fmt == "parquet":
                t = t.select([c for c in cols if c in t.column_names])
        if self.include_paths:
            import pyarrow as pa

            t = t.append_column("path", pa.array([p] * t.num_rows))
        return t


def _read(paths, fmt, exts, include_paths=False, partition_filter=None, file_extensions=None,
          **kw) -> Dataset:
    """``partition_filter``: a ``PathPartitionFilter`` pruning files by partition values;
    ``file_extensions``: overrides the format's default extensions."""
    bases = {}
    if file_extensions is not None:
        exts = ["." + e.lstrip(".") for e in ([file_extensions] if isinstance(file_extensions, str)
                                              else file_extensions)]
    files = _expand_paths(paths, exts, bases)
    if partition_filter is not None:
        files = _filter_partitions(partition_filter, files, bases)
    if not files:
        raise ValueError(f"No input files found to read from paths {paths}")
    return Dataset([("read", _FileRead(f, fmt, kw, include_paths, bases.get(f))) for f in files])


def _file_kw(kw):
    """The file-selection options every read_* accepts (``partition_filter``, ``file_extensions``)."""
    return {k: kw[k] for k in ("partition_filter", "file_extensions") if kw.get(k) is not None}


def _filter_partitions(pf, files, bases):
    """Apply a PathPartitionFilter; its parser's base_dir defaults to each file's read root."""
    from .partitioning import Partitioning, PathPartitionFilter, PathPartitionParser

    scheme = pf.parser.scheme
    if scheme.base_dir:
        return pf(files)
    keep = []
    for f in files:
        parser = PathPartitionParser(Partitioning(scheme.style, bases.get(f, ""), scheme.field_names,
                                                  scheme.field_types))
        keep.extend(PathPartitionFilter(parser, pf._fn)([f]))
    return keep


def _partitioning(p):
    """``partitioning``: "hive" (default), None, or a ``Partitioning`` (HIVE, or DIRECTORY with
    ``field_names``); a base_dir-less HIVE scheme without field checks is the plain "hive" path."""
    if p is None:
        return None
    from .partitioning import Partitioning, PartitionStyle

    if isinstance(p, Partitioning):
        if p.style == PartitionStyle.HIVE and not p.base_dir and not p.field_names and not p.field_types:
            return "hive"
        return p
    style = getattr(p, "value", p)
    if str(style).lower() == "hive":
        return "hive"
    raise ValueError(f"partitioning must be 'hive', None or a Partitioning, got {p!r}")


def read_parquet(paths, *, columns=None, include_paths=False, partitioning="hive", filter=None, **kw) -> Dataset:
    """Parquet files; hive ``col=value`` directories become string columns (reference default
    ``Partitioning("hive")``); ``filter``: a pyarrow filter expression / DNF list."""
    return _read(paths, "parquet", [".parquet"], include_paths, columns=columns, filter=filter,
                 partitioning=_partitioning(partitioning), **_file_kw(kw))


def read_csv(paths, *, include_paths=False, partitioning="hive", parse_options=None, read_options=None,
             convert_options=None, **kw) -> Dataset:
    """CSV files through ``pyarrow.csv`` (``parse_options`` / ``read_options`` / ``convert_options``
    forwarded, e.g. ``ParseOptions(delimiter="\t")``)."""
    return _read(paths, "csv", [".csv"], include_paths, partitioning=_partitioning(partitioning),
                 parse_options=parse_options, read_options=read_options, convert_options=convert_options,
                 **_file_kw(kw))


def read_json(paths, *, include_paths=False, partitioning="hive", parse_options=None, read_options=None,
              **kw) -> Dataset:
    return _read(paths, "json", [".json", ".jsonl"], include_paths, partitioning=_partitioning(partitioning),
                 parse_options=parse_options, read_options=read_options, **_file_kw(kw))


def read_text(paths, *, encoding="utf-8", drop_empty_lines=True, include_paths=False, **kw) -> Dataset:
    return _read(paths, "text", None, include_paths, encoding=encoding, drop_empty_lines=drop_empty_lines,
                 **_file_kw(kw))


def read_numpy(paths, **kw) -> Dataset:
    return _read(paths, "numpy", [".npy"], **_file_kw(kw))


def read_binary_files(paths, *, include_paths=False, **kw) -> Dataset:
    return _read(paths, "binary", None, include_paths, **_file_kw(kw))


def read_images(paths, *, size=None, mode="RGB", include_paths=False, **kw) -> Dataset:
    return _read(paths, "images", [".png", ".jpg", ".jpeg", ".bmp", ".gif", ".tif", ".tiff"], include_paths,
                 size=size, mode=mode, **_file_kw(kw))


def read_datasource(datasource, *, parallelism: int = -1, **read_args) -> Dataset:
    par = parallelism if parallelism > 0 else 2 * _cpus()
    if getattr(datasource, "should_create_reader", lambda: False)():  # legacy Reader-style sources
        tasks = datasource.create_reader(**read_args).get_read_tasks(par)
    else:
        tasks = datasource.get_read_tasks(par, **read_args)
    return Dataset([("read", t) for t in tasks])


class Datasource:
    """Custom datasource (reference ``python/ray/data/datasource/datasource.py``): implement
    ``get_read_tasks(parallelism) -> list of zero-arg callables`` returning blocks. The legacy
    Reader API (``create_reader(**read_args)`` -> an object with ``get_read_tasks`` /
    ``estimate_inmemory_data_size``) is accepted too."""

    def get_read_tasks(self, parallelism: int, **kw):
        raise NotImplementedError

    def get_name(self) -> str:
        name = type(self).__name__
        return name[: -len("Datasource")] if name.endswith("Datasource") and len(name) > 10 else name

    def estimate_inmemory_data_size(self) -> Optional[int]:
        return None

    @property
    def supports_distributed_reads(self) -> bool:
        return True

    def should_create_reader(self) -> bool:
        """True for sources written against the legacy Reader API (they override create_reader)."""
        return type(self).create_reader is not Datasource.create_reader

    def create_reader(self, **read_args):
        return _DatasourceReader(self, read_args)

    def prepare_read(self, parallelism: int, **read_args):
        """Deprecated reference alias of ``get_read_tasks``."""
        return self.get_read_tasks(parallelism, **read_args)


class _DatasourceReader:
    def __init__(self, ds, read_args):
        self._ds, self._args = ds, read_args

    def get_read_tasks(self, parallelism: int):
        return self._ds.get_read_tasks(parallelism, **self._args)

    def estimate_inmemory_data_size(self):
        return self._ds.estimate_inmemory_data_size()
