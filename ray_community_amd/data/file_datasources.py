"""File-based and built-in datasources (reference: python/ray/data/datasource/
file_based_datasource.py, file_meta_provider.py, filename_provider.py and the
``_internal/datasource/*_datasource.py`` family).

``FileBasedDatasource`` is the extension point for custom file formats: subclass it, implement
``_read_stream(f, path) -> Iterator[Block]`` (``f`` an open binary file), and read it with
``ray.data.read_datasource(MyDatasource(paths))``. Files are expanded (directories walked,
globs matched), filtered by extension and by a ``PathPartitionFilter``, and packed into at most
``parallelism`` read tasks of similar byte size; partition fields and (``include_paths``) the file
path are appended to each block.

The concrete sources (Parquet, CSV, JSON, text, NumPy, binary, images, TFRecords, WebDataset,
range, random ints, SQL, torch datasets) reuse the same readers as ``ray.data.read_*``. MongoDB
and BigQuery need client libraries that are not installed: constructing them raises ImportError.
"""
from __future__ import annotations

import os
import uuid
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Tuple, Union

import numpy as np

from .block import BlockAccessor, concat_blocks
from .datasource import ReadTask, Datasink
from .partitioning import FileExtensionFilter, Partitioning, PathPartitionFilter, PathPartitionParser
from .read_api import Datasource, _expand_paths

Block = Any


# ============================================================================ metadata providers
class FileMetadataProvider:
    """Block metadata for a set of files (the size estimate the read-task packing uses)."""

    def __call__(self, paths: List[str], schema=None, *, rows_per_file: Optional[int] = None,
                 file_sizes: Optional[List[Optional[int]]] = None):
        from .block import BlockMetadata

        sizes = [s for s in (file_sizes or []) if s is not None]
        return BlockMetadata(num_rows=rows_per_file * len(paths) if rows_per_file else None,
                             size_bytes=sum(sizes) if sizes else None, schema=schema, input_files=list(paths))


class BaseFileMetadataProvider(FileMetadataProvider):
    def expand_paths(self, paths: List[str], filesystem=None, partitioning=None,
                     ignore_missing_paths: bool = False) -> Iterator[Tuple[str, Optional[int]]]:
        raise NotImplementedError


class DefaultFileMetadataProvider(BaseFileMetadataProvider):
    """Walks directories and stats every file (sizes drive the read-task packing)."""

    def expand_paths(self, paths, filesystem=None, partitioning=None, ignore_missing_paths=False):
        for p in _expand_paths(paths):
            try:
                yield p, os.path.getsize(p)
            except OSError:
                if not ignore_missing_paths:
                    raise FileNotFoundError(p)


class FastFileMetadataProvider(DefaultFileMetadataProvider):
    """Skips the per-file stat (sizes unknown: files are packed by count)."""

    def expand_paths(self, paths, filesystem=None, partitioning=None, ignore_missing_paths=False):
        for p in _expand_paths(paths):
            if not os.path.exists(p) and not ignore_missing_paths:
                raise FileNotFoundError(p)
            if os.path.exists(p):
                yield p, None


class ParquetMetadataProvider(FileMetadataProvider):
    def prefetch_file_metadata(self, fragments, **ray_remote_args):
        return None


DefaultParquetMetadataProvider = ParquetMetadataProvider


# ============================================================================ filename providers
class FilenameProvider:
    """Names the files a file datasink writes (one per block, or one per row for row sinks)."""

    def get_filename_for_block(self, block: Block, task_index: int, block_index: int) -> str:
        raise NotImplementedError

    def get_filename_for_row(self, row: Dict[str, Any], task_index: int, block_index: int,
                             row_index: int) -> str:
        raise NotImplementedError


class _DefaultFilenameProvider(FilenameProvider):
    def __init__(self, dataset_uuid: Optional[str] = None, file_format: Optional[str] = None):
        self._uuid = dataset_uuid or uuid.uuid4().hex[:12]
        self._ext = f".{file_format}" if file_format else ""

    def get_filename_for_block(self, block, task_index, block_index):
        return f"{self._uuid}_{task_index:06d}_{block_index:06d}{self._ext}"

    def get_filename_for_row(self, row, task_index, block_index, row_index):
        return f"{self._uuid}_{task_index:06d}_{block_index:06d}_{row_index:06d}{self._ext}"


class BlockWritePathProvider:
    """Deprecated predecessor of FilenameProvider: the full path of each written block."""

    def __call__(self, base_path: str, *, filesystem=None, dataset_uuid: Optional[str] = None,
                 task_index: Optional[int] = None, block_index: Optional[int] = None,
                 file_format: Optional[str] = None) -> str:
        return self._get_write_path_for_block(base_path, filesystem=filesystem, dataset_uuid=dataset_uuid,
                                              task_index=task_index, block_index=block_index,
                                              file_format=file_format)

    def _get_write_path_for_block(self, base_path, **kw) -> str:
        raise NotImplementedError


class DefaultBlockWritePathProvider(BlockWritePathProvider):
    def _get_write_path_for_block(self, base_path, *, filesystem=None, dataset_uuid=None, task_index=None,
                                  block_index=None, file_format=None):
        return os.path.join(base_path, f"{dataset_uuid}_{task_index:06d}_{block_index:06d}.{file_format}")


# ============================================================================ FileBasedDatasource
class _FileGroupRead:
    """One read task: the files of a group, each through the datasource's ``_read_stream``."""

    def __init__(self, ds: "FileBasedDatasource", files: List[str]):
        self.ds, self.files = ds, files

    def __call__(self):
        blocks = []
        for path in self.files:
            for b in self.ds._read_file_blocks(path):
                if BlockAccessor(b).num_rows():
                    blocks.append(b)
        if not blocks:
            return {}
        return concat_blocks(blocks) if len(blocks) > 1 else blocks[0]


class FileBasedDatasource(Datasource):
    """Subclass and implement ``_read_stream(f, path)`` (or ``_read_file(f, path)`` returning one
    block). ``_FILE_EXTENSIONS`` sets the default extension filter."""

    _FILE_EXTENSIONS: Optional[List[str]] = None
    _NUM_THREADS_PER_TASK = 0

    def __init__(self, paths: Union[str, List[str]], *, filesystem=None, schema=None,
                 open_stream_args: Optional[Dict[str, Any]] = None,
                 meta_provider: Optional[BaseFileMetadataProvider] = None,
                 partition_filter: Optional[PathPartitionFilter] = None,
                 partitioning: Optional[Partitioning] = None, ignore_missing_paths: bool = False,
                 shuffle: Union[str, None] = None, include_paths: bool = False,
                 file_extensions: Optional[List[str]] = None):
        self._paths_in = [paths] if isinstance(paths, str) else list(paths)
        self._schema = schema
        self._partitioning = partitioning
        self._include_paths = include_paths
        self._shuffle = shuffle
        provider = meta_provider or DefaultFileMetadataProvider()
        entries = list(provider.expand_paths(self._paths_in, filesystem, partitioning, ignore_missing_paths))
        if file_extensions is None and self._FILE_EXTENSIONS is not None:
            file_extensions = self._FILE_EXTENSIONS
        if file_extensions is not None:
            keep = set(FileExtensionFilter(file_extensions)([p for p, _ in entries]))
            entries = [(p, s) for p, s in entries if p in keep]
        if partition_filter is not None:
            keep = set(partition_filter([p for p, _ in entries]))
            entries = [(p, s) for p, s in entries if p in keep]
        if not entries and not ignore_missing_paths:
            raise ValueError(f"No input files found to read from paths {self._paths_in}")
        if shuffle == "files":
            rng = np.random.default_rng()
            entries = [entries[i] for i in rng.permutation(len(entries))]
        self._entries = entries
        self._base = self._base_dir()

    def _base_dir(self) -> str:
        if self._partitioning is not None and self._partitioning.base_dir:
            return self._partitioning.base_dir
        dirs = [p for p in self._paths_in if os.path.isdir(p)]
        return dirs[0] if len(dirs) == 1 else ""

    # -- subclass API
    def _read_stream(self, f, path: str) -> Iterator[Block]:
        yield self._read_file(f, path)

    def _read_file(self, f, path: str) -> Block:
        raise NotImplementedError("FileBasedDatasource subclasses implement _read_stream or _read_file")

    def _open_input_source(self, path: str):
        return open(path, "rb")

    # -- machinery
    def _read_file_blocks(self, path: str) -> Iterator[Block]:
        fields: Dict[str, Any] = {}
        if self._partitioning is not None:
            scheme = self._partitioning
            if not scheme.base_dir and self._base:
                scheme = Partitioning(scheme.style, self._base, scheme.field_names, scheme.field_types)
            fields = PathPartitionParser(scheme)(path)
        with self._open_input_source(path) as f:
            for b in self._read_stream(f, path):
                yield self._decorate(b, path, fields)

    def _decorate(self, block: Block, path: str, fields: Dict[str, Any]) -> Block:
        if not fields and not self._include_paths:
            return block
        n = BlockAccessor(block).num_rows()
        extra = dict(fields)
        if self._include_paths:
            extra["path"] = path
        if hasattr(block, "append_column"):  # arrow
            import pyarrow as pa

            for k, v in extra.items():
                if k not in block.column_names:
                    block = block.append_column(k, pa.array([v] * n))
            return block
        if hasattr(block, "assign"):  # pandas
            return block.assign(**{k: [v] * n for k, v in extra.items() if k not in block.columns})
        out = dict(block)
        for k, v in extra.items():
            out.setdefault(k, np.asarray([v] * n, dtype=object if isinstance(v, str) else None))
        return out

    def _paths(self) -> List[str]:
        return [p for p, _ in self._entries]

    def _file_sizes(self) -> List[Optional[int]]:
        return [s for _, s in self._entries]

    def estimate_inmemory_data_size(self) -> Optional[int]:
        sizes = self._file_sizes()
        if any(s is None for s in sizes):
            return None
        return int(sum(sizes))

    def get_read_tasks(self, parallelism: int, **kw) -> List[ReadTask]:
        """At most ``parallelism`` tasks, files packed greedily by size (largest first into the
        lightest task), file order kept inside each task."""
        n = len(self._entries)
        if n == 0:
            return []
        k = max(1, min(parallelism if parallelism > 0 else n, n))
        groups: List[List[int]] = [[] for _ in range(k)]
        loads = [0] * k
        order = sorted(range(n), key=lambda i: -(self._entries[i][1] or 1))
        for i in order:
            j = loads.index(min(loads))
            groups[j].append(i)
            loads[j] += self._entries[i][1] or 1
        tasks = []
        meta = FileMetadataProvider()
        for g in groups:
            if not g:
                continue
            g.sort()
            files = [self._entries[i][0] for i in g]
            tasks.append(ReadTask(_FileGroupRead(self, files),
                                  meta(files, self._schema, file_sizes=[self._entries[i][1] for i in g])))
        return tasks

    @property
    def supports_distributed_reads(self) -> bool:
        return True


# ============================================================================ concrete formats
def _arrow_kw(kw, names):
    return {k: kw[k] for k in names if kw.get(k) is not None}


class ParquetBaseDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["parquet"]

    def __init__(self, paths, *, columns=None, filter=None, **kw):
        self._columns, self._filter = columns, filter
        super().__init__(paths, **kw)

    def _read_stream(self, f, path):
        import pyarrow.parquet as pq

        yield pq.read_table(f, columns=self._columns, filters=self._filter)


class ParquetDatasource(ParquetBaseDatasource):
    pass


class CSVDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["csv"]

    def __init__(self, paths, *, arrow_csv_args: Optional[Dict] = None, **kw):
        self._args = dict(arrow_csv_args or {})
        super().__init__(paths, **kw)

    def _read_stream(self, f, path):
        import pyarrow.csv as pcsv

        yield pcsv.read_csv(f, **_arrow_kw(self._args, ("read_options", "parse_options", "convert_options")))


class JSONDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["json", "jsonl"]

    def __init__(self, paths, *, arrow_json_args: Optional[Dict] = None, **kw):
        self._args = dict(arrow_json_args or {})
        super().__init__(paths, **kw)

    def _read_stream(self, f, path):
        import pyarrow.json as pj

        yield pj.read_json(f, **_arrow_kw(self._args, ("read_options", "parse_options")))


class TextDatasource(FileBasedDatasource):
    def __init__(self, paths, *, drop_empty_lines: bool = True, encoding: str = "utf-8", **kw):
        self._drop, self._enc = drop_empty_lines, encoding
        super().__init__(paths, **kw)

    def _read_stream(self, f, path):
        lines = f.read().decode(self._enc).splitlines()
        if self._drop:
            lines = [l for l in lines if l.strip()]
        yield {"text": np.asarray(lines, dtype=object)}


class NumpyDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["npy"]

    def __init__(self, paths, *, numpy_load_args: Optional[Dict] = None, **kw):
        self._args = dict(numpy_load_args or {})
        self._args["allow_pickle"] = False  # never unpickle file contents
        super().__init__(paths, **kw)

    def _read_stream(self, f, path):
        yield {"data": np.load(f, **self._args)}


class BinaryDatasource(FileBasedDatasource):
    def _read_stream(self, f, path):
        a = np.empty(1, dtype=object)
        a[0] = f.read()
        yield {"bytes": a}


class ImageDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["png", "jpg", "jpeg", "tif", "tiff", "bmp", "gif"]

    def __init__(self, paths, *, size: Optional[Tuple[int, int]] = None, mode: Optional[str] = None, **kw):
        self._size, self._mode = size, mode
        super().__init__(paths, **kw)

    def _read_stream(self, f, path):
        from PIL import Image  # optional dependency

        img = Image.open(f)
        if self._mode:
            img = img.convert(self._mode)
        if self._size:
            img = img.resize(self._size[::-1])
        yield {"image": np.asarray(img)[None]}


class TFRecordDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["tfrecords", "tfrecord"]

    def __init__(self, paths, *, verify_checksums: bool = False, **kw):
        self._verify = verify_checksums
        super().__init__(paths, **kw)

    def _open_input_source(self, path):
        import contextlib

        return contextlib.nullcontext(path)

    def _read_stream(self, path, _):
        from .datasource import _TFRecordRead

        yield _TFRecordRead(path, self._verify)()


class WebDatasetDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["tar"]

    def __init__(self, paths, *, decoder=True, suffixes: Optional[List[str]] = None, **kw):
        self._decoder, self._suffixes = decoder, suffixes
        super().__init__(paths, **kw)

    def _open_input_source(self, path):
        import contextlib

        return contextlib.nullcontext(path)

    def _read_stream(self, path, _):
        from .datasource import _WebDatasetRead

        yield _WebDatasetRead(path, self._decoder, self._suffixes)()


# ============================================================================ non-file sources
class RangeDatasource(Datasource):
    def __init__(self, n: int, block_format: str = "arrow", tensor_shape: Tuple = (1,), column_name: str = "id"):
        self._n, self._fmt, self._shape, self._col = int(n), block_format, tuple(tensor_shape), column_name

    def estimate_inmemory_data_size(self):
        return 8 * self._n * int(np.prod(self._shape)) if self._fmt == "tensor" else 8 * self._n

    def get_read_tasks(self, parallelism: int, **kw):
        k = max(1, min(parallelism, self._n) if parallelism > 0 else 1)
        bounds = np.linspace(0, self._n, k + 1).astype(np.int64)
        out = []
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            if hi > lo:
                out.append(ReadTask(_RangeBlock(int(lo), int(hi), self._fmt, self._shape, self._col)))
        return out


class _RangeBlock:
    def __init__(self, lo, hi, fmt, shape, col):
        self.lo, self.hi, self.fmt, self.shape, self.col = lo, hi, fmt, shape, col

    def __call__(self):
        ids = np.arange(self.lo, self.hi, dtype=np.int64)
        if self.fmt == "tensor":
            return {"data": np.broadcast_to(ids.reshape((-1,) + (1,) * len(self.shape)),
                                            (len(ids),) + self.shape).copy()}
        if self.fmt == "arrow":
            import pyarrow as pa

            return pa.table({self.col: ids})
        return {self.col: ids}


class RandomIntRowDatasource(Datasource):
    """``n`` rows of ``num_columns`` random int64 columns ``c_0 .. c_{k-1}`` in [0, 2^63)."""

    def __init__(self, n: int, num_columns: int):
        self._n, self._k = int(n), int(num_columns)

    def estimate_inmemory_data_size(self):
        return 8 * self._n * self._k

    def get_read_tasks(self, parallelism: int, **kw):
        k = max(1, min(parallelism, self._n) if parallelism > 0 else 1)
        bounds = np.linspace(0, self._n, k + 1).astype(np.int64)
        return [ReadTask(_RandomInts(int(hi - lo), self._k, i)) for i, (lo, hi) in
                enumerate(zip(bounds[:-1], bounds[1:])) if hi > lo]


class _RandomInts:
    def __init__(self, n, k, seed):
        self.n, self.k, self.seed = n, k, seed

    def __call__(self):
        rng = np.random.default_rng()
        return {f"c_{j}": rng.integers(0, np.iinfo(np.int64).max, self.n, dtype=np.int64) for j in range(self.k)}


class SQLDatasource(Datasource):
    def __init__(self, sql: str, connection_factory: Callable[[], Any]):
        self.sql, self.connection_factory = sql, connection_factory

    def get_read_tasks(self, parallelism: int, **kw):
        from .datasource import _sql_read_tasks

        return [ReadTask(t) for t in _sql_read_tasks(self.sql, self.connection_factory, max(1, parallelism))]


class TorchDatasource(Datasource):
    """A map-style ``torch.utils.data.Dataset``: items become rows of an ``item`` column."""

    def __init__(self, dataset):
        self._dataset = dataset

    def get_read_tasks(self, parallelism: int, **kw):
        n = len(self._dataset)
        k = max(1, min(parallelism, n) if parallelism > 0 else 1)
        bounds = np.linspace(0, n, k + 1).astype(np.int64)
        return [ReadTask(_TorchSlice(self._dataset, int(lo), int(hi))) for lo, hi in
                zip(bounds[:-1], bounds[1:]) if hi > lo]


class _TorchSlice:
    def __init__(self, ds, lo, hi):
        self.ds, self.lo, self.hi = ds, lo, hi

    def __call__(self):
        a = np.empty(self.hi - self.lo, dtype=object)
        for i in range(self.lo, self.hi):
            a[i - self.lo] = self.ds[i]
        return {"item": a}


class _ClientLibraryDatasource(Datasource):
    _LIB = ""

    def __init__(self, *a, **k):
        raise ImportError(f"{type(self).__name__} needs {self._LIB}, which is not installed in this environment")


class MongoDatasource(_ClientLibraryDatasource):
    _LIB = "pymongo / pymongoarrow"


class BigQueryDatasource(_ClientLibraryDatasource):
    _LIB = "google-cloud-bigquery"


class DummyOutputDatasink(Datasink):
    """Counts the rows written (the reference's test sink); ``num_ok`` / ``num_failed`` track
    completed and failed writes."""

    def __init__(self):
        self.rows_written = 0
        self.num_ok = 0
        self.num_failed = 0
        self.enabled = True

    def write(self, blocks, ctx):
        if not self.enabled:
            raise ValueError("disabled")
        return sum(BlockAccessor(b).num_rows() for b in blocks)

    def on_write_complete(self, write_results):
        self.rows_written += sum(int(r or 0) for r in write_results)
        self.num_ok += 1

    def on_write_failed(self, error):
        self.num_failed += 1


Reader = Datasource  # the legacy Reader protocol: get_read_tasks + estimate_inmemory_data_size
Connection = Any  # DB-API 2 connection type (read_sql's connection_factory returns one)

__all__ = ["FileMetadataProvider", "BaseFileMetadataProvider", "DefaultFileMetadataProvider",
           "FastFileMetadataProvider", "ParquetMetadataProvider", "DefaultParquetMetadataProvider",
           "FilenameProvider", "BlockWritePathProvider", "DefaultBlockWritePathProvider", "FileBasedDatasource",
           "ParquetBaseDatasource", "ParquetDatasource", "CSVDatasource", "JSONDatasource", "TextDatasource",
           "NumpyDatasource", "BinaryDatasource", "ImageDatasource", "TFRecordDatasource", "WebDatasetDatasource",
           "RangeDatasource", "RandomIntRowDatasource", "SQLDatasource", "TorchDatasource", "MongoDatasource",
           "BigQueryDatasource", "DummyOutputDatasink", "Reader", "Connection"]
