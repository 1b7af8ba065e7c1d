"""Ray Data equivalent (reference: ``python/ray/data``)."""
from .aggregate import AbsMax, AggregateFn, Count, Max, Mean, Min, Std, Sum, Unique
from .block import BlockAccessor
from .context import DataContext, DatasetContext
from .dataset import ActorPoolStrategy, Dataset, MaterializedDataset, Schema, TaskPoolStrategy
from .grouped_data import GroupedData
from .iterator import DataIterator
from .context import ExecutionOptions
from ._internal.resource_manager import ExecutionResources
from .block import BlockMetadata
from .datasource import (BlockBasedFileDatasink, Datasink, ReadTask, RowBasedFileDatasink, from_arrow_refs, from_dask,
                         from_mars, from_modin, from_pandas_refs, from_spark, from_tf, read_bigquery,
                         read_databricks_tables, read_mongo, read_parquet_bulk, read_sql, read_tfrecords,
                         read_webdataset)
from .preprocessors import Preprocessor

DatasetIterator = DataIterator
NodeIdStr = str


def set_progress_bars(enabled: bool) -> bool:
    """Enable/disable progress bars; returns the previous setting."""
    ctx = DataContext.get_current()
    old = ctx.enable_progress_bars
    ctx.enable_progress_bars = bool(enabled)
    return old
from .random_access_dataset import RandomAccessDataset
from .read_api import (Datasource, from_arrow, from_huggingface, from_items, from_numpy, from_numpy_refs, from_pandas,
                       from_torch, range, range_tensor, read_binary_files, read_csv, read_datasource, read_images,
                       read_json, read_numpy, read_parquet, read_text)

__all__ = ["Dataset", "MaterializedDataset", "DataIterator", "GroupedData", "ActorPoolStrategy", "TaskPoolStrategy",
           "DataContext", "DatasetContext", "Schema", "BlockAccessor", "range", "range_tensor", "from_items",
           "from_numpy", "from_numpy_refs", "from_pandas", "from_arrow", "from_torch", "from_huggingface",
           "read_parquet", "read_csv", "read_json", "read_text", "read_numpy", "read_binary_files", "read_images",
           "read_datasource", "Datasource", "AggregateFn", "Count", "Sum", "Min", "Max", "Mean", "Std", "AbsMax",
           "Unique", "Datasink", "read_sql", "read_webdataset", "read_tfrecords", "read_parquet_bulk",
           "from_pandas_refs", "from_arrow_refs", "RandomAccessDataset", "ExecutionOptions", "ExecutionResources", "BlockMetadata",
           "ReadTask", "RowBasedFileDatasink", "BlockBasedFileDatasink", "DatasetIterator", "NodeIdStr",
           "set_progress_bars", "Preprocessor", "from_dask", "from_mars", "from_modin", "from_spark", "from_tf",
           "read_mongo", "read_bigquery", "read_databricks_tables"]
