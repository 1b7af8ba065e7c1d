"""Dataset (reference: ``python/ray/data/dataset.py``): lazy, block-based, streaming."""
from __future__ import annotations

import collections
import inspect
import itertools
import math
import os
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Tuple, Union

import numpy as np

from .block import BlockAccessor, concat_blocks, normalize_block
from ._internal import execution as X

_MAP_KINDS = {"map_batches", "map", "flat_map", "filter", "add_column", "drop_columns", "select_columns",
              "rename_columns"}


def _cpus():
    try:
        from .._private.worker import cluster_resources, is_initialized

        if is_initialized():
            return max(1, int(cluster_resources().get("CPU", 1)))
    except Exception:
        pass
    return os.cpu_count() or 1


def _ensure_init():
    from .._private import worker as w

    if not w.is_initialized():
        w.init()


class ActorPoolStrategy:
    """Actor-pool compute: ``size`` (fixed) or ``min_size`` / ``max_size`` (the streaming executor
    scales the pool between them on queue depth and idleness). Reference:
    ``python/ray/data/_internal/compute.py`` ``ActorPoolStrategy``."""

    def __init__(self, size: Optional[int] = None, min_size: Optional[int] = None, max_size: Optional[int] = None,
                 max_tasks_in_flight_per_actor: int = 4):
        if size is not None and (min_size is not None or max_size is not None):
            raise ValueError("min_size and max_size cannot be set at the same time as `size`")
        if size is not None:
            min_size = max_size = size
        self.min_size = int(min_size or 1)
        self.max_size = int(max_size) if max_size is not None else (self.min_size if min_size is not None else
                                                                     self.min_size)
        if self.max_size < self.min_size:
            raise ValueError("min_size must be <= max_size")
        self.size = self.max_size
        self.max_tasks_in_flight_per_actor = max_tasks_in_flight_per_actor


class TaskPoolStrategy:
    def __init__(self, size: Optional[int] = None):
        self.size = size


class Schema:
    def __init__(self, names, types):
        self.names = list(names)
        self.types = list(types)

    def __repr__(self):
        return "Schema(" + ", ".join(f"{n}: {t}" for n, t in zip(self.names, self.types)) + ")"

    def __eq__(self, o):
        return isinstance(o, Schema) and o.names == self.names


class Dataset:
    def __init__(self, inputs: List, ops: Optional[List[Dict]] = None, name: Optional[str] = None):
        self._inputs = inputs
        self._ops = list(ops or [])
        self._name = name
        self._materialized: Optional[List[Tuple[Any, Any]]] = None

    def __getstate__(self):
        # the plan and any materialised refs travel; the last execution's executor / resource
        # manager (threads, locks) stay with the process that ran it
        st = dict(self.__dict__)
        for k in ("_executor", "_exec_rm"):
            st.pop(k, None)
        return st

    # ------------------------------------------------------------------ plan helpers
    def _with(self, op) -> "Dataset":
        return Dataset(self._inputs, self._ops + [op], self._name)

    def _iter_refs(self) -> Iterator[Tuple[Any, Any]]:
        _ensure_init()
        if self._materialized is not None:
            return iter(self._materialized)
        from .context import DataContext
        from ._internal.resource_manager import ResourceManager

        ctx = DataContext.get_current()
        rm = ResourceManager.from_context(ctx)
        ctx.last_execution_stats = rm
        self._exec_rm = rm
        window = max(2, 2 * _cpus())
        from ._internal import streaming_executor as SE

        ordered = bool(ctx.execution_options.preserve_order)
        ex = SE.StreamingExecutor([], rm, window)
        ops: List = [SE.InputOp(self._inputs, ordered, rm, rm.register("Read", cpu=1))]

        def task_op(chain):
            opts = _task_opts(chain)
            caps = [o.get("concurrency") for o in chain if isinstance(o.get("concurrency"), int)]
            name = "->".join(_op_name(o) for o in chain)
            st = rm.register(name, cpu=opts.get("num_cpus", 1) or 0, gpu=opts.get("num_gpus", 0) or 0,
                             concurrency_cap=min(caps) if caps else None)
            return SE.TaskMapOp(name, chain, opts, ordered, rm, st)

        from ._internal import logical_optimizer as LO

        logical, rules = LO.push_down_limits(self._ops, getattr(ctx, "enable_limit_pushdown", True))
        fuse = getattr(ctx, "enable_operator_fusion", True)
        stages = LO.plan_stages(logical, fuse)
        if fuse and any(st[0] == "actor" and st[2] or st[0] == "task" and len(st[1]) > 1 for st in stages):
            rules = rules + ["OperatorFusion"]
        self._plan_info = {"logical": LO.describe([("task", [o]) if o["kind"] in _MAP_KINDS and
                                                    o.get("compute") != "actors" else
                                                    (("actor", o, []) if o["kind"] in _MAP_KINDS else
                                                     (("limit", o["n"]) if o["kind"] == "limit" else ("alltoall", o)))
                                                    for o in self._ops], _op_name),
                           "optimized": LO.describe(stages, _op_name), "rules": rules}
        for st in stages:
            if st[0] == "task":
                ops.append(task_op(st[1]))
            elif st[0] == "actor":  # actor pool operator (autoscaling between min and max)
                op, pre = st[1], st[2]
                mif = op.get("max_tasks_in_flight_per_actor", 4)
                name = "->".join([_op_name(o) for o in pre] + [_op_name(op)]) + "(actors)"
                caps = [o.get("concurrency") for o in pre if isinstance(o.get("concurrency"), int)]
                st_rm = rm.register(name, concurrency_cap=min([op["max_size"] * mif] + caps))
                ops.append(SE.ActorPoolMapOp(name, op, op["actor_opts"], op["min_size"], op["max_size"], mif,
                                             ctx.actor_pool_idle_timeout_s, ordered, rm, st_rm, pre_ops=pre))
            elif st[0] == "limit":
                ops.append(SE.LimitOp(st[1], ordered, ex))
            elif st[0] == "nary":
                op = st[1]
                if op["kind"] == "union":
                    ops.append(SE.UnionOp(op["others"], ordered, window))
                else:
                    ops.append(SE.ZipOp(op["other"], ordered, window))
            else:
                ops.append(SE.AllToAllOp(st[1].get("name", "AllToAll"), st[1]["fn"], ordered))
        ex.__init__(ops, rm, window)
        self._executor = ex
        return ex.start().iter_outputs()

    def _refs(self) -> List[Tuple[Any, Any]]:
        if self._materialized is None:
            self._materialized = list(self._iter_refs())
            self._inputs = [("ref", b, m) for b, m in self._materialized]
            self._ops = []
        return self._materialized

    def _metas(self):
        from .._private.worker import get

        refs = self._refs()
        return get([m for _, m in refs]) if refs else []

    # ------------------------------------------------------------------ transforms
    def map_batches(self, fn, *, batch_size: Union[int, None, str] = "default", compute=None,
                    batch_format: Optional[str] = "default", zero_copy_batch: bool = False, fn_args=None,
                    fn_kwargs=None, fn_constructor_args=None, fn_constructor_kwargs=None, num_cpus=None,
                    num_gpus=None, concurrency=None, **ray_remote_args) -> "Dataset":
        if batch_size == "default":
            batch_size = 1024 if not inspect.isclass(fn) else 1024
        op = {"kind": "map_batches", "fn": fn, "batch_size": batch_size, "batch_format": batch_format,
              "fn_args": tuple(fn_args or ()), "fn_kwargs": dict(fn_kwargs or {}), "num_cpus": num_cpus,
              "num_gpus": num_gpus, "ray_remote_args": ray_remote_args}
        return self._with(_compute(op, fn, compute, concurrency, fn_constructor_args, fn_constructor_kwargs, num_cpus,
                                   num_gpus, ray_remote_args))

    def map(self, fn, *, compute=None, fn_args=None, fn_kwargs=None, fn_constructor_args=None,
            fn_constructor_kwargs=None, num_cpus=None, num_gpus=None, concurrency=None, **ray_remote_args):
        op = {"kind": "map", "fn": fn, "fn_args": tuple(fn_args or ()), "fn_kwargs": dict(fn_kwargs or {}),
              "num_cpus": num_cpus, "num_gpus": num_gpus, "ray_remote_args": ray_remote_args}
        return self._with(_compute(op, fn, compute, concurrency, fn_constructor_args, fn_constructor_kwargs, num_cpus,
                                   num_gpus, ray_remote_args))

    def flat_map(self, fn, *, compute=None, fn_args=None, fn_kwargs=None, fn_constructor_args=None,
                 fn_constructor_kwargs=None, num_cpus=None, num_gpus=None, concurrency=None, **ray_remote_args):
        op = {"kind": "flat_map", "fn": fn, "fn_args": tuple(fn_args or ()), "fn_kwargs": dict(fn_kwargs or {}),
              "num_cpus": num_cpus, "num_gpus": num_gpus, "ray_remote_args": ray_remote_args}
        return self._with(_compute(op, fn, compute, concurrency, fn_constructor_args, fn_constructor_kwargs, num_cpus,
                                   num_gpus, ray_remote_args))

    def filter(self, fn=None, *, expr: Optional[str] = None, compute=None, concurrency=None, **kw):
        op = {"kind": "filter", "fn": fn, "expr": expr}
        return self._with(_compute(op, fn, compute, concurrency, None, None, None, None, kw))

    def add_column(self, col: str, fn: Callable, *, batch_format: str = "pandas", **kw):
        return self._with({"kind": "add_column", "col": col, "fn": fn, "batch_format": batch_format})

    def drop_columns(self, cols: List[str], **kw):
        return self._with({"kind": "drop_columns", "cols": list(cols)})

    def select_columns(self, cols: List[str], **kw):
        return self._with({"kind": "select_columns", "cols": list(cols) if not isinstance(cols, str) else [cols]})

    def rename_columns(self, names: Dict[str, str], **kw):
        return self._with({"kind": "rename_columns", "mapping": dict(names)})

    def limit(self, limit: int) -> "Dataset":
        return self._with({"kind": "limit", "n": int(limit)})

    def repartition(self, num_blocks: int, *, shuffle: bool = False, seed=None) -> "Dataset":
        def fn(refs):
            return _repartition(refs, num_blocks, shuffle, seed)

        return self._with({"kind": "alltoall", "fn": fn})

    def random_shuffle(self, *, seed: Optional[int] = None, num_blocks: Optional[int] = None, **kw) -> "Dataset":
        def fn(refs):
            k = num_blocks or max(1, len(refs))
            return _repartition(refs, k, True, seed)

        return self._with({"kind": "alltoall", "fn": fn})

    def randomize_block_order(self, *, seed: Optional[int] = None) -> "Dataset":
        def fn(refs):
            rng = np.random.default_rng(seed)
            idx = rng.permutation(len(refs))
            return [refs[i] for i in idx]

        return self._with({"kind": "alltoall", "fn": fn})

    def sort(self, key: Union[str, List[str]], descending: Union[bool, List[bool]] = False,
             boundaries: Optional[List] = None) -> "Dataset":
        """Sort by one or more columns (lexicographic; ``descending`` per column or for all).
        Rows are range-partitioned on the first column -- at sampled quantiles, or at the given
        ``boundaries`` (one output block per range) -- and each partition sorts by every key."""
        keys = [key] if isinstance(key, str) else list(key)
        if not keys:
            raise ValueError("sort needs at least one key")
        desc = [bool(descending)] * len(keys) if isinstance(descending, bool) else [bool(d) for d in descending]
        if len(desc) != len(keys):
            raise ValueError(f"descending has {len(desc)} entries for {len(keys)} keys")

        def fn(refs):
            return _sort(refs, keys, desc, boundaries)

        return self._with({"kind": "alltoall", "fn": fn})

    def groupby(self, key: Union[str, List[str], None]) -> "GroupedData":
        from .grouped_data import GroupedData

        return GroupedData(self, key)

    def union(self, *others: "Dataset") -> "Dataset":
        """Streaming union (``_internal/streaming_executor.py::UnionOp``): the other datasets
        execute concurrently with this one; with ``preserve_order`` the result is this dataset's
        rows, then each other's in argument order."""
        return self._with({"kind": "union", "others": list(others), "name": "Union"})

    def zip(self, other: "Dataset") -> "Dataset":
        """Streaming zip (``ZipOp``): rows are aligned across the two block streams as they
        arrive (no materialisation of either side); both must have the same row count."""
        return self._with({"kind": "zip", "other": other, "name": "Zip"})

    def random_sample(self, fraction: float, *, seed: Optional[int] = None) -> "Dataset":
        def sample(batch, fraction=fraction, seed=seed):
            n = len(next(iter(batch.values()))) if batch else 0
            rng = np.random.default_rng(seed)
            mask = rng.random(n) < fraction
            return {k: v[mask] for k, v in batch.items()}

        return self.map_batches(sample, batch_format="numpy", batch_size=None)

    # ------------------------------------------------------------------ splits
    def split(self, n: int, *, equal: bool = False, locality_hints=None) -> List["MaterializedDataset"]:
        refs = self._refs()
        metas = self._metas()
        total = sum(m["num_rows"] for m in metas)
        if equal:
            per = total // n
            sizes = [per] * n
        else:
            sizes = [total // n + (1 if i < total % n else 0) for i in range(n)]
        parts = _repartition_to_sizes(refs, sizes, metas)
        return [MaterializedDataset([p]) for p in parts]

    def split_at_indices(self, indices: List[int]) -> List["MaterializedDataset"]:
        metas = self._metas()
        total = sum(m["num_rows"] for m in metas)
        bounds = [0] + list(indices) + [total]
        sizes = [max(0, b - a) for a, b in zip(bounds[:-1], bounds[1:])]
        parts = _repartition_to_sizes(self._refs(), sizes, metas)
        return [MaterializedDataset([p]) for p in parts]

    def split_proportionately(self, proportions: List[float]):
        total = self.count()
        idx = []
        acc = 0
        for p in proportions:
            acc += int(total * p)
            idx.append(acc)
        return self.split_at_indices(idx)

    def train_test_split(self, test_size: Union[int, float], *, shuffle: bool = False, seed=None):
        ds = self.random_shuffle(seed=seed) if shuffle else self
        total = ds.count()
        n_test = int(test_size) if isinstance(test_size, int) else int(math.ceil(total * test_size))
        a, b = ds.split_at_indices([total - n_test])
        return a, b

    def streaming_split(self, n: int, *, equal: bool = False, locality_hints=None) -> List["DataIterator"]:
        """``n`` iterators over ONE streaming execution of this dataset, coordinated by a split
        actor (``_internal/stream_split.py``): returns immediately, executes lazily, re-executes
        every epoch (all ``n`` iterators must start it), ``equal=True`` gives every iterator
        exactly ``count // n`` rows. Reference: ``python/ray/data/dataset.py:1141``."""
        _ensure_init()
        from ._internal.stream_split import streaming_split

        return streaming_split(self, n, equal, locality_hints)

    # ------------------------------------------------------------------ consumption
    def iterator(self) -> "DataIterator":
        from .iterator import DataIterator

        return DataIterator(self)

    def iter_batches(self, **kw):
        return self.iterator().iter_batches(**kw)

    def iter_torch_batches(self, **kw):
        return self.iterator().iter_torch_batches(**kw)

    def iter_rows(self, **kw) -> Iterator[Dict]:
        from .._private.worker import get

        for b, _ in self._iter_refs():
            yield from BlockAccessor(get(b)).iter_rows()

    def take(self, limit: int = 20) -> List[Dict]:
        out = []
        for r in self.limit(limit).iter_rows():
            out.append(r)
            if len(out) >= limit:
                break
        return out

    def take_all(self, limit: Optional[int] = None) -> List[Dict]:
        out = list(self.iter_rows())
        if limit is not None and len(out) > limit:
            raise ValueError(f"The dataset has more than the given limit of {limit} records.")
        return out

    def take_batch(self, batch_size: int = 20, *, batch_format: str = "default"):
        for b in self.limit(batch_size).iter_batches(batch_size=batch_size, batch_format=batch_format):
            return b
        return {}

    def show(self, limit: int = 20):
        for r in self.take(limit):
            print(r)

    def count(self) -> int:
        return int(sum(m["num_rows"] for m in self._metas()))

    def schema(self, fetch_if_missing: bool = True):
        from .._private.worker import get

        for b, m in self._iter_refs():
            blk = get(b)
            acc = BlockAccessor(blk)
            if acc.num_rows() == 0 and not acc.column_names():
                continue
            if hasattr(blk, "schema"):
                s = blk.schema
                return Schema(s.names, [str(t) for t in s.types])
            return Schema(list(blk.keys()), [f"{v.dtype}{list(v.shape[1:]) if v.ndim > 1 else ''}"
                                             for v in blk.values()])
        return None

    def columns(self, fetch_if_missing: bool = True):
        s = self.schema()
        return s.names if s else []

    def num_blocks(self) -> int:
        return len(self._refs())

    def size_bytes(self) -> int:
        return int(sum(m["size_bytes"] for m in self._metas()))

    def materialize(self) -> "MaterializedDataset":
        return MaterializedDataset(self._refs())

    def to_pandas(self, limit: Optional[int] = None):
        import pandas as pd

        from .._private.worker import get

        dfs = [BlockAccessor(get(b)).to_pandas() for b, _ in self._iter_refs()]
        df = pd.concat(dfs, ignore_index=True) if dfs else pd.DataFrame()
        if limit is not None and len(df) > limit:
            raise ValueError(f"the dataset has more than the given limit of {limit} rows")
        return df

    def to_numpy_refs(self, *, column=None):
        from .._private.worker import get, put

        return [put(BlockAccessor(get(b)).to_numpy() if column is None else BlockAccessor(get(b)).to_numpy()[column])
                for b, _ in self._refs()]

    def to_arrow_refs(self):
        from .._private.worker import get, put

        return [put(BlockAccessor(get(b)).to_arrow()) for b, _ in self._refs()]

    def to_pandas_refs(self):
        from .._private.worker import get, put

        return [put(BlockAccessor(get(b)).to_pandas()) for b, _ in self._refs()]

    def get_internal_block_refs(self):
        return [b for b, _ in self._refs()]

    def to_torch(self, *, label_column=None, feature_columns=None, batch_size=1, **kw):
        import torch

        class _It(torch.utils.data.IterableDataset):
            def __iter__(_s):
                for b in self.iter_torch_batches(batch_size=batch_size):
                    if label_column:
                        y = b.pop(label_column)
                        cols = feature_columns or list(b)
                        yield torch.stack([b[c].float() for c in cols], dim=1), y
                    else:
                        yield b

        return _It()

    # ------------------------------------------------------------------ lineage
    def has_serializable_lineage(self) -> bool:
        """True when the dataset can be re-created from its plan alone: every input is a read
        task (not an in-memory block ref) and nothing is materialised (reference
        ``Dataset.has_serializable_lineage``)."""
        if self._materialized is not None:
            return False
        return all(x[0] != "ref" for x in self._inputs) and all(
            not isinstance(o.get(k), Dataset) or o[k].has_serializable_lineage()
            for o in self._ops for k in ("other",)) and all(
            d.has_serializable_lineage() for o in self._ops for d in (o.get("others") or ()))

    def serialize_lineage(self) -> bytes:
        """The dataset's plan (read tasks + operators), without any block refs: a bytes object a
        later session (or another cluster) turns back into the same dataset with
        ``Dataset.deserialize_lineage`` and re-executes."""
        if not self.has_serializable_lineage():
            raise ValueError("Lineage-based serialization is not supported for this dataset: it has in-memory "
                             "(from_* / materialized) inputs; only read_* datasets carry their full lineage")
        import cloudpickle

        return cloudpickle.dumps(Dataset(self._inputs, self._ops, self._name))

    @staticmethod
    def deserialize_lineage(serialized_ds: bytes) -> "Dataset":
        import cloudpickle

        ds = cloudpickle.loads(serialized_ds)
        if not isinstance(ds, Dataset):
            raise TypeError("not a serialized Dataset lineage")
        return ds

    # ------------------------------------------------------------------ other frameworks
    def _absent(self, what: str, lib: str):
        raise ImportError(f"Dataset.{what} needs {lib}, which is not installed in this MI355X image")

    def to_tf(self, *a, **k):
        self._absent("to_tf", "TensorFlow")

    def iter_tf_batches(self, *a, **k):
        self._absent("iter_tf_batches", "TensorFlow")

    def to_dask(self, *a, **k):
        self._absent("to_dask", "dask")

    def to_mars(self, *a, **k):
        self._absent("to_mars", "mars")

    def to_modin(self, *a, **k):
        self._absent("to_modin", "modin")

    def to_spark(self, *a, **k):
        self._absent("to_spark", "raydp / pyspark")

    def write_bigquery(self, *a, **k):
        self._absent("write_bigquery", "google-cloud-bigquery")

    def write_mongo(self, *a, **k):
        self._absent("write_mongo", "pymongo")

    def write_datasource(self, datasource, *, ray_remote_args=None, **write_args):
        """Legacy write API (reference ``write_datasource``, superseded by ``write_datasink``): a
        datasource object with ``write(blocks, ctx, **write_args)`` (and optional
        ``on_write_complete`` / ``on_write_failed``) receives the blocks, one write task per block."""
        from .._private.worker import get
        from ..remote_function import RemoteFunction

        def _write_one(block, i):
            return datasource.write([block], {"task_idx": i}, **write_args)

        rf = RemoteFunction(_write_one, dict(ray_remote_args or {}, num_cpus=(ray_remote_args or {}).get("num_cpus", 1)))
        try:
            results = get([rf.remote(b, i) for i, (b, _) in enumerate(self._iter_refs())])
        except Exception as e:
            if hasattr(datasource, "on_write_failed"):
                datasource.on_write_failed([], e)
            raise
        if hasattr(datasource, "on_write_complete"):
            datasource.on_write_complete(results)
        return results

    # ------------------------------------------------------------------ aggregations
    def aggregate(self, *aggs):
        return self.groupby(None).aggregate(*aggs).take(1)[0]

    def sum(self, on=None, ignore_nulls=True):
        return self._agg1("sum", on)

    def min(self, on=None, ignore_nulls=True):
        return self._agg1("min", on)

    def max(self, on=None, ignore_nulls=True):
        return self._agg1("max", on)

    def mean(self, on=None, ignore_nulls=True):
        return self._agg1("mean", on)

    def std(self, on=None, ddof=1, ignore_nulls=True):
        from .aggregate import Std

        r = self.aggregate(Std(on, ddof=ddof))
        return list(r.values())[0]

    def unique(self, column: str) -> List:
        vals = set()
        for b in self.select_columns([column]).iter_batches(batch_format="numpy"):
            vals.update(np.unique(b[column]).tolist())
        return list(vals)

    def _agg1(self, how, on):
        from . import aggregate as A

        cls = {"sum": A.Sum, "min": A.Min, "max": A.Max, "mean": A.Mean}[how]
        if on is None:
            on = self.columns()[0]
        if isinstance(on, list):
            r = self.aggregate(*[cls(c) for c in on])
            return r
        r = self.aggregate(cls(on))
        return list(r.values())[0]

    # ------------------------------------------------------------------ writes
    def write_parquet(self, path: str, *, partition_cols: Optional[List[str]] = None, **kw):
        """``partition_cols``: hive layout ``path/col=value/...`` with those columns moved into
        the directory names (reference ``Dataset.write_parquet``); ``read_parquet`` restores them."""
        self._sized(kw)._write(path, "parquet", partition_cols=list(partition_cols or []),
                             filename_provider=kw.get("filename_provider"))

    def write_csv(self, path: str, **kw):
        self._sized(kw)._write(path, "csv", filename_provider=kw.get("filename_provider"))

    def write_json(self, path: str, **kw):
        self._sized(kw)._write(path, "json", filename_provider=kw.get("filename_provider"))

    def write_numpy(self, path: str, *, column: str = "data", **kw):
        self._sized(kw)._write(path, "npy", column=column, filename_provider=kw.get("filename_provider"))

    def _sized(self, kw) -> "Dataset":
        """``min_rows_per_file`` / ``num_rows_per_file`` (reference writers): coalesce blocks so
        every written file holds at least that many rows (one file per block otherwise)."""
        n = kw.get("min_rows_per_file") or kw.get("num_rows_per_file")
        if not n:
            return self
        total = self.count()
        return self.repartition(max(1, total // int(n)))

    def write_datasink(self, datasink, *, ray_remote_args=None, concurrency=None):
        from .datasource import write_datasink

        write_datasink(self, datasink, ray_remote_args=ray_remote_args, concurrency=concurrency)

    def write_sql(self, sql: str, connection_factory, **kw):
        from .datasource import SQLDatasink

        self.write_datasink(SQLDatasink(sql, connection_factory))

    def write_images(self, path: str, column: str, file_format: str = "png", **kw):
        from .datasource import ImageDatasink

        self.write_datasink(ImageDatasink(path, column, file_format))

    def write_webdataset(self, path: str, **kw):
        from .datasource import WebDatasetDatasink

        self.write_datasink(WebDatasetDatasink(path))

    def write_tfrecords(self, path: str, **kw):
        from .datasource import TFRecordDatasink

        self.write_datasink(TFRecordDatasink(path))

    def to_random_access_dataset(self, key: str, num_workers: Optional[int] = None):
        from .random_access_dataset import RandomAccessDataset

        return RandomAccessDataset(self, key, num_workers or 4)

    def input_files(self) -> List[str]:
        """Files the dataset's read stage reads (empty for in-memory datasets)."""
        out = []
        for st in self._inputs or []:
            fn = st[1] if isinstance(st, tuple) and len(st) > 1 and st[0] == "read" else None
            p = getattr(fn, "path", None)
            if isinstance(p, str) and p not in out:
                out.append(p)
        return out

    def copy(self) -> "Dataset":
        import copy as _copy

        return _copy.copy(self)

    def _write(self, path, fmt, column=None, partition_cols=None, filename_provider=None):
        """One file per block; ``filename_provider`` (a ``FilenameProvider``) names them
        (``get_filename_for_block(block, task_index, block_index)``), else ``{index:06d}.{fmt}``."""
        from .._private.worker import get

        os.makedirs(path, exist_ok=True)
        w = X._remote_fn(_write_block, {"num_cpus": 1})
        refs = [w.remote(b, path, i, fmt, column, partition_cols, filename_provider)[0]
                for i, (b, _) in enumerate(self._refs())]
        get(refs)

    # ------------------------------------------------------------------ misc
    def stats(self) -> str:
        ms = self._metas()
        out = (f"Dataset: {len(ms)} blocks, {sum(m['num_rows'] for m in ms)} rows, "
               f"{sum(m['size_bytes'] for m in ms) / 2**20:.2f} MiB")
        pi = getattr(self, "_plan_info", None)
        if pi is not None:
            out += f"\n  Logical plan: {pi['logical']}"
            out += f"\n  Optimized plan: {pi['optimized']}"
            if pi["rules"]:
                out += f"\n  Optimizer rules applied: {', '.join(pi['rules'])}"
        rm = getattr(self, "_exec_rm", None)
        if rm is not None:
            st = rm.stats()
            for o in st["ops"]:
                out += (f"\n  Operator {o['name']}: {o['tasks']} tasks, peak {o['peak_running']} concurrent, "
                        f"backpressured {o['backpressured']}x, {o['output_bytes'] / 2**20:.2f} MiB out")
        ex = getattr(self, "_executor", None)
        if ex is not None:
            for name, o in ex.stats.items():
                if "peak_pool_size" in o:
                    out += (f"\n  Actor pool {name}: peak {o['peak_pool_size']} actors, {o['scale_ups']} scale-ups, "
                            f"{o['scale_downs']} scale-downs")
        return out

    def _execution_stats(self) -> Optional[Dict]:
        """Resource-manager counters of this dataset's last execution (limits, peaks, per op)."""
        rm = getattr(self, "_exec_rm", None)
        if rm is None:
            return None
        rm.poll()
        return rm.stats()

    def __repr__(self):
        return f"Dataset(num_ops={len(self._ops)}, materialized={self._materialized is not None})"

    def __len__(self):
        raise AttributeError("Use ds.count() to compute the length of a distributed Dataset.")

    def __iter__(self):
        raise TypeError("`Dataset` objects aren't iterable. To iterate records, call `ds.iter_rows()` or "
                        "`ds.iter_batches()`.")

    def context(self):
        from .context import DataContext

        return DataContext.get_current()


class MaterializedDataset(Dataset):
    def __init__(self, refs):
        super().__init__([("ref", b, m) for b, m in refs])
        self._materialized = list(refs)


# ---------------------------------------------------------------------------------- helpers
def _op_name(op) -> str:
    fn = op.get("fn")
    n = getattr(fn, "__name__", None) or type(fn).__name__ if fn is not None else None
    k = {"map_batches": "MapBatches", "map": "Map", "flat_map": "FlatMap", "filter": "Filter"}.get(op["kind"], op["kind"])
    return f"{k}({n})" if n else k


def _compute(op, fn, compute, concurrency, ctor_args, ctor_kwargs, num_cpus, num_gpus, ray_remote_args):
    is_class = inspect.isclass(fn)
    use_actors = is_class or isinstance(compute, ActorPoolStrategy) or compute == "actors"
    if use_actors:
        size = 1
        lo = hi = None
        if isinstance(compute, ActorPoolStrategy):
            lo, hi = compute.min_size, compute.max_size
            op["max_tasks_in_flight_per_actor"] = compute.max_tasks_in_flight_per_actor
        elif concurrency is not None:
            if isinstance(concurrency, tuple):
                lo, hi = int(concurrency[0]), int(concurrency[-1])
            else:
                lo = hi = int(concurrency)
        op["compute"] = "actors"
        op["min_size"] = max(1, lo or size)
        op["max_size"] = max(op["min_size"], hi or op["min_size"])
        op["pool_size"] = op["max_size"]
        opts = {"num_cpus": 1 if num_cpus is None else num_cpus}
        if num_gpus:
            opts["num_gpus"] = num_gpus
        for k, v in (ray_remote_args or {}).items():
            if k in ("resources", "memory", "scheduling_strategy", "runtime_env", "max_restarts"):
                opts[k] = v
        op["actor_opts"] = opts
        op["fn_constructor_args"] = tuple(ctor_args or ())
        op["fn_constructor_kwargs"] = dict(ctor_kwargs or {})
        if not is_class:
            f = fn

            class _Wrap:
                def __init__(self):
                    pass

                def __call__(self, *a, **k):
                    return f(*a, **k)

            op["fn"] = _Wrap
    else:
        op["compute"] = "tasks"
        if isinstance(concurrency, int):
            op["concurrency"] = concurrency  # task-pool concurrency cap (backpressure policy)
    return op


def _task_opts(ops):
    cpus = max([o.get("num_cpus") or 0 for o in ops] + [0]) or 1
    gpus = max([o.get("num_gpus") or 0 for o in ops] + [0])
    opts = {"num_cpus": cpus}
    if gpus:
        opts["num_gpus"] = gpus
    for o in ops:
        for k, v in (o.get("ray_remote_args") or {}).items():
            if k in ("resources", "memory", "scheduling_strategy", "runtime_env", "max_retries"):
                opts[k] = v
    return opts


def _repartition(refs, k, shuffle, seed):
    from .._private.worker import get

    if not refs:
        return []
    metas = get([m for _, m in refs])
    if shuffle:
        base = 0 if seed is None else int(seed)
        args = [(k, base * 1000003 + i if seed is not None else None) for i in range(len(refs))]
        return X.exchange(refs, k, X._split_random, args, X._reduce_concat,
                          [{"shuffle_seed": (base + j) if seed is not None else int(np.random.randint(1 << 30))}
                           for j in range(k)])
    total = sum(m["num_rows"] for m in metas)
    sizes = [total // k + (1 if i < total % k else 0) for i in range(k)]
    return _repartition_to_sizes(refs, sizes, metas)


def _repartition_to_sizes(refs, sizes, metas=None):
    from .._private.worker import get

    if metas is None:
        metas = get([m for _, m in refs])
    bounds = [0]
    for s in sizes:
        bounds.append(bounds[-1] + s)
    starts = []
    acc = 0
    for m in metas:
        starts.append(acc)
        acc += m["num_rows"]
    return X.exchange(refs, len(sizes), X._split_by_ranges, [(s, bounds) for s in starts], X._reduce_concat,
                      [{} for _ in sizes])


def _sort(refs, keys, desc, boundaries=None):
    from .._private.worker import get

    if not refs:
        return []
    key, descending = keys[0], desc[0]
    if boundaries is not None:  # user ranges on the first key: one output block per range
        bounds = np.sort(np.asarray(list(boundaries)))
        k = len(bounds) + 1
    else:
        k = len(refs)
        sample_fn = X._remote_fn(_sample_keys, {"num_cpus": 1})
        samples = get([sample_fn.remote(b, key)[0] for b, _ in refs])
        allk = np.concatenate([s for s in samples if len(s)]) if any(len(s) for s in samples) else np.array([])
        if len(allk) == 0:
            return refs
        bounds = np.sort(np.quantile(np.sort(allk), np.linspace(0, 1, k + 1)[1:-1])) if k > 1 else np.array([])
    sort_key = key if len(keys) == 1 else list(keys)
    sort_desc = descending if len(keys) == 1 else list(desc)
    return X.exchange(refs, k, X._split_by_key_bounds, [(key, bounds, descending) for _ in refs],
                      X._reduce_concat, [{"sort_key": sort_key, "descending": sort_desc} for _ in range(k)])


def _sample_keys(block, key):
    d = BlockAccessor(block).to_numpy()
    if key not in d or len(d[key]) == 0:
        return np.array([]), {}
    v = d[key]
    idx = np.random.default_rng(0).choice(len(v), size=min(len(v), 64), replace=False)
    return v[idx], {}


def _pa_table(df):
    import pyarrow as pa

    return pa.Table.from_pandas(df, preserve_index=False)


def _write_block(block, path, i, fmt, column, partition_cols=None, filename_provider=None):
    acc = BlockAccessor(block)
    if acc.num_rows() == 0:
        return None, {}
    name = filename_provider.get_filename_for_block(block, i, 0) if filename_provider is not None else None
    fn = os.path.join(path, name or f"{i:06d}.{fmt}")
    if fmt == "parquet" and partition_cols:
        import pyarrow.parquet as pq

        df = acc.to_pandas()
        missing = [c for c in partition_cols if c not in df.columns]
        if missing:
            raise ValueError(f"partition_cols {missing} are not columns of the dataset")
        out = []
        for key, part in df.groupby(partition_cols, sort=True, dropna=False):
            key = key if isinstance(key, tuple) else (key,)
            d = os.path.join(path, *[f"{c}={v}" for c, v in zip(partition_cols, key)])
            os.makedirs(d, exist_ok=True)
            f = os.path.join(d, name or f"{i:06d}.parquet")
            pq.write_table(_pa_table(part.drop(columns=partition_cols).reset_index(drop=True)), f)
            out.append(f)
        return out, {}
    if fmt == "parquet":
        import pyarrow.parquet as pq

        pq.write_table(acc.to_arrow(), fn)
    elif fmt == "csv":
        acc.to_pandas().to_csv(fn, index=False)
    elif fmt == "json":
        acc.to_pandas().to_json(fn, orient="records", lines=True)
    elif fmt == "npy":
        np.save(fn, acc.to_numpy()[column])
    return fn, {}
