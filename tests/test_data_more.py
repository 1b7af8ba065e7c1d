"""More Data behaviour (reference test models: python/ray/data/tests/test_streaming_split.py,
test_map.py (fn_constructor_args, batch_format, zero-copy), test_consumption.py (iter_rows,
take_batch, show, schema), test_formats.py (from_pandas/from_arrow/from_numpy round trips),
test_all_to_all.py (aggregations), test_size_estimation.py (size_bytes))."""
import threading

import numpy as np
import pandas as pd
import pytest

import ray_community_amd as ray
from ray_community_amd import data


@pytest.fixture
def ray4():
    ray.init(num_cpus=4, log_to_driver=False)
    yield
    ray.shutdown()


def test_streaming_split_feeds_concurrent_consumers_disjointly(ray4):
    ds = data.range(1000, override_num_blocks=20)
    its = ds.streaming_split(2, equal=True)
    got = [[], []]

    def consume(i):
        for b in its[i].iter_batches(batch_size=50):
            got[i].extend(int(x) for x in b["id"])

    ts = [threading.Thread(target=consume, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert len(got[0]) == len(got[1]) == 500
    assert sorted(got[0] + got[1]) == list(range(1000))


def test_callable_class_with_constructor_args(ray4):
    class AddK:
        def __init__(self, k, scale=1):
            self.k = k * scale

        def __call__(self, batch):
            batch["id"] = batch["id"] + self.k
            return batch

    ds = data.range(40).map_batches(AddK, fn_constructor_args=(10,), fn_constructor_kwargs={"scale": 2},
                                    concurrency=2, batch_size=8)
    assert sorted(r["id"] for r in ds.take_all()) == [i + 20 for i in range(40)]


def test_batch_formats_round_trip(ray4):
    ds = data.from_items([{"a": i, "b": float(i) * 0.5} for i in range(10)])
    pdf = ds.map_batches(lambda df: df.assign(c=df["a"] * 2), batch_format="pandas").to_pandas()
    assert list(pdf["c"]) == [2 * i for i in range(10)]
    npb = ds.map_batches(lambda b: {"s": b["a"] + b["b"]}, batch_format="numpy").take_batch(10)
    assert isinstance(npb["s"], np.ndarray) and np.allclose(npb["s"], np.arange(10) * 1.5)
    pa = pytest.importorskip("pyarrow")
    tb = pa.table({"x": list(range(6))})
    back = data.from_arrow(tb).map_batches(lambda t: t, batch_format="pyarrow").to_pandas()
    assert list(back["x"]) == list(range(6))


def test_from_pandas_numpy_and_schema(ray4):
    df = pd.DataFrame({"x": np.arange(8), "y": np.arange(8) * 1.5})
    ds = data.from_pandas([df.iloc[:4], df.iloc[4:]])
    assert ds.count() == 8
    names = ds.schema().names
    assert set(names) == {"x", "y"}
    arr = data.from_numpy(np.ones((6, 3), dtype=np.float32))
    b = arr.take_batch(6)
    assert b["data"].shape == (6, 3)
    rows = list(ds.iter_rows())
    assert rows[3]["x"] == 3 and rows[5]["y"] == 7.5


def test_global_aggregations(ray4):
    ds = data.from_items([{"v": float(i)} for i in range(1, 11)])
    assert ds.sum("v") == 55.0
    assert ds.min("v") == 1.0 and ds.max("v") == 10.0
    assert ds.mean("v") == 5.5
    assert abs(ds.std("v") - np.std(np.arange(1, 11), ddof=1)) < 1e-9


def test_materialize_stats_and_size(ray4):
    ds = data.range(100).map(lambda r: {"id": r["id"], "sq": r["id"] ** 2}).materialize()
    assert ds.count() == 100
    assert ds.size_bytes() > 0
    s = ds.stats()
    assert isinstance(s, str) and s
    assert ds.take(3) == [{"id": 0, "sq": 0}, {"id": 1, "sq": 1}, {"id": 2, "sq": 4}]


def test_add_column_and_rename(ray4):
    ds = data.range(5).add_column("double", lambda df: df["id"] * 2)
    assert [r["double"] for r in ds.take_all()] == [0, 2, 4, 6, 8]
    ds2 = ds.rename_columns({"double": "d"})
    assert set(ds2.columns()) == {"id", "d"}
