"""More Data sources and sinks (reference: ``python/ray/data/datasource/*``, ``_internal/datasource/*``).

* ``Datasink`` + ``Dataset.write_datasink``: user sinks get ``on_write_start`` -> ``write`` per
  block (in a task per block, with a ``TaskContext``) -> ``on_write_complete(results)`` (or
  ``on_write_failed``), as ``datasource/datasink.py``.
* SQL (DB-API 2): ``read_sql(sql, connection_factory)`` sharded with LIMIT/OFFSET when the row
  count is known, ``Dataset.write_sql("INSERT ... VALUES (?, ?)", connection_factory)`` with one
  ``executemany`` per block (``sql_datasource.py`` / ``sql_datasink.py``).
* WebDataset tar shards: ``read_webdataset`` groups the members of a tar by sample key
  (basename up to the first dot) into one row per sample with one column per extension,
  decoding ``.jpg/.png``, ``.json``, ``.txt``, ``.cls``, ``.npy``; ``write_webdataset`` writes one
  shard per block (``webdataset_datasource.py``).
* TFRecords: ``read_tfrecords`` / ``write_tfrecords`` over ``tf.train.Example`` records with
  masked CRC32C framing -- the Example message is built from a descriptor at import (protobuf is
  installed, TensorFlow is not), so files interoperate with TF readers/writers.
* ``write_images`` (PIL), ``from_pandas_refs`` / ``from_arrow_refs``, ``read_parquet_bulk``.
"""
from __future__ import annotations

import io
import json
import os
import struct
import tarfile
from typing import Any, Callable, Dict, Iterable, List, Optional

import numpy as np

from .block import BlockAccessor, rows_to_block
from .dataset import Dataset


# ============================================================================ Datasink
class TaskContext:
    def __init__(self, task_idx: int):
        self.task_idx = task_idx
        self.kwargs: Dict[str, Any] = {}


class Datasink:
    """Write-side extension point. ``write`` runs in a task per block and returns any picklable
    value; ``on_write_complete`` gets the list of those values on the driver."""

    def on_write_start(self) -> None:
        pass

    def write(self, blocks: Iterable[Any], ctx: TaskContext) -> Any:
        raise NotImplementedError

    def on_write_complete(self, write_results: List[Any]) -> None:
        pass

    def on_write_failed(self, error: Exception) -> None:
        pass

    def get_name(self) -> str:
        n = type(self).__name__
        return n[: -len("Datasink")] if n.endswith("Datasink") and len(n) > 8 else n

    @property
    def supports_distributed_writes(self) -> bool:
        return True

    @property
    def num_rows_per_write(self) -> Optional[int]:
        return None


def _sink_task(sink, block, idx):
    return sink.write([block], TaskContext(idx))


def write_datasink(ds: Dataset, datasink: Datasink, *, ray_remote_args: Optional[dict] = None,
                   concurrency: Optional[int] = None) -> None:
    from .._private.worker import get
    from ._internal import execution as X

    datasink.on_write_start()
    try:
        if datasink.num_rows_per_write:
            ds = ds.repartition(max(1, -(-ds.count() // datasink.num_rows_per_write)))
        if datasink.supports_distributed_writes:
            fn = X._remote_fn(_sink_task, dict({"num_cpus": 1}, **(ray_remote_args or {}), num_returns=1))
            refs = [fn.remote(datasink, b, i) for i, (b, _) in enumerate(ds._refs())]
            results = get(refs)
        else:
            blocks = [get(b) for b, _ in ds._refs()]
            results = [datasink.write(blocks, TaskContext(0))]
    except Exception as e:  # noqa
        datasink.on_write_failed(e)
        raise
    datasink.on_write_complete(results)


# ============================================================================ SQL
class _SQLRead:
    def __init__(self, sql, factory, limit=None, offset=None):
        self.sql, self.factory, self.limit, self.offset = sql, factory, limit, offset

    def __call__(self):
        q = self.sql if self.limit is None else f"SELECT * FROM ({self.sql}) LIMIT {self.limit} OFFSET {self.offset}"
        conn = self.factory()
        try:
            cur = conn.cursor()
            cur.execute(q)
            cols = [d[0] for d in cur.description]
            rows = cur.fetchall()
        finally:
            conn.close()
        if not rows:
            return {c: np.asarray([], dtype=object) for c in cols}
        return rows_to_block([dict(zip(cols, r)) for r in rows])


def read_sql(sql: str, connection_factory: Callable[[], Any], *, parallelism: int = -1,
             override_num_blocks: Optional[int] = None, **kw) -> Dataset:
    """Rows of a query. With more than one block the query is sharded as
    ``SELECT * FROM (sql) LIMIT n OFFSET k`` over ``SELECT COUNT(*) FROM (sql)`` rows (the query
    must be deterministic for that, as in the reference)."""
    k = override_num_blocks or (parallelism if parallelism and parallelism > 0 else 1)
    return Dataset([("read", t) for t in _sql_read_tasks(sql, connection_factory, k)])


def _sql_read_tasks(sql: str, connection_factory: Callable[[], Any], k: int) -> List[_SQLRead]:
    if k <= 1:
        return [_SQLRead(sql, connection_factory)]
    conn = connection_factory()
    try:
        cur = conn.cursor()
        cur.execute(f"SELECT COUNT(*) FROM ({sql})")
        n = int(cur.fetchone()[0])
    finally:
        conn.close()
    k = max(1, min(k, n))
    bounds = [n * i // k for i in range(k + 1)]
    return [_SQLRead(sql, connection_factory, bounds[i + 1] - bounds[i], bounds[i]) for i in range(k)]


class SQLDatasink(Datasink):
    def __init__(self, sql: str, connection_factory: Callable[[], Any]):
        self.sql, self.factory = sql, connection_factory

    def write(self, blocks, ctx):
        conn = self.factory()
        n = 0
        try:
            cur = conn.cursor()
            for b in blocks:
                rows = [tuple(_py(v) for v in r.values()) for r in BlockAccessor(b).iter_rows()]
                if rows:
                    cur.executemany(self.sql, rows)
                    n += len(rows)
            conn.commit()
        finally:
            conn.close()
        return n


def _py(v):
    return v.item() if isinstance(v, np.generic) else v


# ============================================================================ images
class ImageDatasink(Datasink):
    def __init__(self, path: str, column: str, file_format: str = "png"):
        self.path, self.column, self.fmt = path, column, file_format

    def on_write_start(self):
        os.makedirs(self.path, exist_ok=True)

    def write(self, blocks, ctx):
        from PIL import Image

        n = 0
        for b in blocks:
            imgs = BlockAccessor(b).to_numpy()[self.column]
            for j, img in enumerate(imgs):
                a = np.asarray(img)
                if a.dtype != np.uint8:
                    a = np.clip(a, 0, 255).astype(np.uint8)
                Image.fromarray(a).save(os.path.join(self.path, f"{ctx.task_idx:06d}_{j:06d}.{self.fmt}"))
                n += 1
        return n


# ============================================================================ WebDataset
_DECODERS = {
    "json": lambda b: json.loads(b.decode("utf-8")),
    "txt": lambda b: b.decode("utf-8"),
    "cls": lambda b: int(b.decode("utf-8").strip()),
    "npy": lambda b: np.load(io.BytesIO(b), allow_pickle=False),
}


def _decode(ext, data, decode):
    if not decode:
        return data
    e = ext.lower().rsplit(".", 1)[-1]
    if e in ("jpg", "jpeg", "png", "bmp", "ppm", "tif", "tiff"):
        from PIL import Image

        return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    fn = _DECODERS.get(e)
    return fn(data) if fn else data


def _encode(ext, v):
    e = ext.lower().rsplit(".", 1)[-1]
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if e in ("jpg", "jpeg", "png"):
        from PIL import Image

        buf = io.BytesIO()
        Image.fromarray(np.asarray(v, dtype=np.uint8)).save(buf, format="PNG" if e == "png" else "JPEG")
        return buf.getvalue()
    if e == "json":
        return json.dumps(v if not isinstance(v, np.ndarray) else v.tolist()).encode()
    if e == "npy":
        buf = io.BytesIO()
        np.save(buf, np.asarray(v), allow_pickle=False)
        return buf.getvalue()
    return str(_py(v)).encode()


class _WebDatasetRead:
    def __init__(self, path, decode, suffixes):
        self.path, self.decode, self.suffixes = path, decode, suffixes

    def __call__(self):
        samples: Dict[str, dict] = {}
        order = []
        with tarfile.open(self.path, "r") as tf:
            for m in tf:
                if not m.isfile():
                    continue
                base = os.path.basename(m.name)
                if "." not in base:
                    continue
                key, ext = base.split(".", 1)
                key = os.path.join(os.path.dirname(m.name), key)
                if self.suffixes and not any(ext.endswith(s) for s in self.suffixes):
                    continue
                data = tf.extractfile(m).read()
                if key not in samples:
                    samples[key] = {"__key__": key}
                    order.append(key)
                samples[key][ext] = _decode(ext, data, self.decode)
        rows = [samples[k] for k in order]
        return rows_to_block(rows) if rows else {"__key__": np.asarray([], dtype=object)}


def read_webdataset(paths, *, decoder=True, suffixes: Optional[List[str]] = None, **kw) -> Dataset:
    from .read_api import _expand_paths

    files = _expand_paths(paths, [".tar"])
    if not files:
        raise ValueError(f"No input files found to read from paths {paths}")
    return Dataset([("read", _WebDatasetRead(f, bool(decoder), suffixes)) for f in files])


class WebDatasetDatasink(Datasink):
    def __init__(self, path: str):
        self.path = path

    def on_write_start(self):
        os.makedirs(self.path, exist_ok=True)

    def write(self, blocks, ctx):
        fn = os.path.join(self.path, f"{ctx.task_idx:06d}.tar")
        n = 0
        with tarfile.open(fn, "w") as tf:
            for b in blocks:
                for j, row in enumerate(BlockAccessor(b).iter_rows()):
                    key = str(row.get("__key__", f"{ctx.task_idx:06d}_{j:06d}"))
                    for col, v in row.items():
                        if col == "__key__":
                            continue
                        data = _encode(col, v)
                        info = tarfile.TarInfo(f"{key}.{col}")
                        info.size = len(data)
                        tf.addfile(info, io.BytesIO(data))
                    n += 1
        return n


# ============================================================================ TFRecords
_EXAMPLE = None


def _example_cls():
    """``tf.train.Example`` built from a descriptor (same field numbers as
    tensorflow/core/example/{example,feature}.proto), so records are wire-compatible with TF."""
    global _EXAMPLE
    if _EXAMPLE is not None:
        return _EXAMPLE
    from google.protobuf import descriptor_pb2, descriptor_pool
    try:
        from google.protobuf import message_factory

        get_cls = getattr(message_factory, "GetMessageClass", None)
    except ImportError:  # pragma: no cover
        get_cls = None
    fdp = descriptor_pb2.FileDescriptorProto(name="rca_tf_example.proto", package="tensorflow", syntax="proto3")
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=()):
        m = fdp.message_type.add(name=name)
        for fname, num, typ, label, tname, oneof in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
            if oneof is not None:
                f.oneof_index = oneof
        return m

    rep, opt = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, F.TYPE_BYTES, rep, None, None)])
    m = msg("FloatList", [("value", 1, F.TYPE_FLOAT, rep, None, None)])
    m.field[0].options.packed = True
    m = msg("Int64List", [("value", 1, F.TYPE_INT64, rep, None, None)])
    m.field[0].options.packed = True
    m = msg("Feature", [("bytes_list", 1, F.TYPE_MESSAGE, opt, ".tensorflow.BytesList", 0),
                        ("float_list", 2, F.TYPE_MESSAGE, opt, ".tensorflow.FloatList", 0),
                        ("int64_list", 3, F.TYPE_MESSAGE, opt, ".tensorflow.Int64List", 0)])
    m.oneof_decl.add(name="kind")
    feats = fdp.message_type.add(name="Features")
    entry = feats.nested_type.add(name="FeatureEntry")
    entry.options.map_entry = True
    entry.field.add(name="key", number=1, type=F.TYPE_STRING, label=opt)
    entry.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=opt, type_name=".tensorflow.Feature")
    feats.field.add(name="feature", number=1, type=F.TYPE_MESSAGE, label=rep,
                    type_name=".tensorflow.Features.FeatureEntry")
    msg("Example", [("features", 1, F.TYPE_MESSAGE, opt, ".tensorflow.Features", None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    desc = pool.FindMessageTypeByName("tensorflow.Example")
    if get_cls is not None:
        _EXAMPLE = get_cls(desc)
    else:  # pragma: no cover  (older protobuf)
        from google.protobuf import reflection

        _EXAMPLE = reflection.message_factory.MessageFactory(pool).GetPrototype(desc)
    return _EXAMPLE


def _crc32c_table():
    poly = 0x82F63B78
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


_CRC_T = None


def _crc32c(data: bytes) -> int:
    global _CRC_T
    if _CRC_T is None:
        _CRC_T = _crc32c_table()
    t = _CRC_T
    c = 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = _crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _tfrecord_iter(path, verify=False):
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                return
            (n,) = struct.unpack("<Q", hdr[:8])
            if verify and struct.unpack("<I", hdr[8:])[0] != _masked_crc(hdr[:8]):
                raise ValueError(f"{path}: corrupt TFRecord length")
            data = f.read(n)
            crc = f.read(4)
            if verify and struct.unpack("<I", crc)[0] != _masked_crc(data):
                raise ValueError(f"{path}: corrupt TFRecord payload")
            yield data


def _feature_value(feat):
    kind = feat.WhichOneof("kind")
    if kind is None:
        return None
    vals = list(getattr(feat, kind).value)
    return vals[0] if len(vals) == 1 else vals


class _TFRecordRead:
    def __init__(self, path, verify):
        self.path, self.verify = path, verify

    def __call__(self):
        Example = _example_cls()
        rows = []
        for rec in _tfrecord_iter(self.path, self.verify):
            ex = Example()
            ex.ParseFromString(rec)
            rows.append({k: _feature_value(v) for k, v in ex.features.feature.items()})
        return rows_to_block(rows) if rows else {}


def read_tfrecords(paths, *, verify_checksums: bool = False, **kw) -> Dataset:
    from .read_api import _expand_paths

    files = _expand_paths(paths, None)
    if not files:
        raise ValueError(f"No input files found to read from paths {paths}")
    return Dataset([("read", _TFRecordRead(f, verify_checksums)) for f in files])


def _set_feature(feat, v):
    if isinstance(v, np.ndarray):
        v = v.reshape(-1).tolist()
    vals = v if isinstance(v, (list, tuple)) else [v]
    vals = [_py(x) for x in vals]
    if not vals:
        feat.bytes_list.value.extend([])
    elif all(isinstance(x, (bytes, bytearray)) for x in vals):
        feat.bytes_list.value.extend([bytes(x) for x in vals])
    elif all(isinstance(x, str) for x in vals):
        feat.bytes_list.value.extend([x.encode() for x in vals])
    elif all(isinstance(x, (bool, int)) for x in vals):
        feat.int64_list.value.extend([int(x) for x in vals])
    else:
        feat.float_list.value.extend([float(x) for x in vals])


class TFRecordDatasink(Datasink):
    def __init__(self, path: str):
        self.path = path

    def on_write_start(self):
        os.makedirs(self.path, exist_ok=True)

    def write(self, blocks, ctx):
        Example = _example_cls()
        fn = os.path.join(self.path, f"{ctx.task_idx:06d}.tfrecords")
        n = 0
        with open(fn, "wb") as f:
            for b in blocks:
                for row in BlockAccessor(b).iter_rows():
                    ex = Example()
                    for k, v in row.items():
                        _set_feature(ex.features.feature[k], v)
                    data = ex.SerializeToString()
                    hdr = struct.pack("<Q", len(data))
                    f.write(hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data)))
                    n += 1
        return n


# ============================================================================ refs / aliases
def from_pandas_refs(refs) -> Dataset:
    from .._private.worker import get
    from .read_api import from_pandas

    return from_pandas(get(list(refs) if isinstance(refs, (list, tuple)) else [refs]))


def from_arrow_refs(refs) -> Dataset:
    from .._private.worker import get
    from .read_api import from_arrow

    return from_arrow(get(list(refs) if isinstance(refs, (list, tuple)) else [refs]))


def read_parquet_bulk(paths, *, columns=None, **kw) -> Dataset:
    from .read_api import read_parquet

    return read_parquet(paths, columns=columns, **kw)


# ============================================================================ file datasinks / ReadTask
class ReadTask:
    """A read unit for ``Datasource.get_read_tasks``: a zero-arg callable producing blocks plus its
    metadata (reference ``datasource/datasource.py``). Returning a list/iterator of blocks is
    allowed; they are concatenated into one block."""

    def __init__(self, read_fn: Callable[[], Iterable[Any]], metadata: Any = None):
        self._read_fn = read_fn
        self.metadata = metadata

    def __call__(self):
        from .block import concat_blocks

        out = self._read_fn()
        if isinstance(out, (dict,)) or hasattr(out, "num_rows") or hasattr(out, "columns"):
            return out
        blocks = list(out)
        return concat_blocks(blocks) if len(blocks) != 1 else blocks[0]


class _FileDatasink(Datasink):
    def __init__(self, path: str, *, file_format: str = "bin", **kw):
        self.path, self.file_format = path, file_format

    def on_write_start(self):
        os.makedirs(self.path, exist_ok=True)


class RowBasedFileDatasink(_FileDatasink):
    """One file per ROW: subclasses implement ``write_row_to_file(row, file)``."""

    def write_row_to_file(self, row: Dict[str, Any], file):
        raise NotImplementedError

    def write(self, blocks, ctx):
        n = 0
        for b in blocks:
            for j, row in enumerate(BlockAccessor(b).iter_rows()):
                with open(os.path.join(self.path, f"{ctx.task_idx:06d}_{j:06d}.{self.file_format}"), "wb") as f:
                    self.write_row_to_file(row, f)
                n += 1
        return n


class BlockBasedFileDatasink(_FileDatasink):
    """One file per BLOCK: subclasses implement ``write_block_to_file(block_accessor, file)``."""

    def write_block_to_file(self, block: BlockAccessor, file):
        raise NotImplementedError

    def write(self, blocks, ctx):
        n = 0
        for j, b in enumerate(blocks):
            acc = BlockAccessor(b)
            if acc.num_rows() == 0:
                continue
            with open(os.path.join(self.path, f"{ctx.task_idx:06d}_{j:06d}.{self.file_format}"), "wb") as f:
                self.write_block_to_file(acc, f)
            n += acc.num_rows()
        return n


def _absent(lib):
    def f(*a, **k):
        raise ImportError(f"{lib} is not installed in this environment; convert to pandas/arrow/numpy first")
    return f


from_dask = _absent("dask")
from_mars = _absent("mars")
from_modin = _absent("modin")
from_spark = _absent("pyspark")
from_tf = _absent("tensorflow")
read_mongo = _absent("pymongo")
read_bigquery = _absent("google-cloud-bigquery")
read_databricks_tables = _absent("databricks-sql-connector")


# the datasource / partitioning / filename-provider classes live in their own modules; this module
# is the ``ray.data.datasource`` import path for all of them (reference datasource/__init__.py)
from .file_datasources import *  # noqa: E402,F401,F403
from .file_datasources import __all__ as _file_all  # noqa: E402
from .partitioning import (FileExtensionFilter, PartitionStyle, Partitioning, PathPartitionFilter,  # noqa: E402,F401
                           PathPartitionParser)
from .read_api import Datasource  # noqa: E402,F401
