"""Tensor columns (reference: python/ray/data/extensions, air/util/tensor_extensions; tests
python/ray/data/tests/test_tensor.py): fixed-shape ndarray columns keep their row shape through
Arrow blocks, pandas batches, the object store and Parquet files."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import ray_community_amd as ray
from ray_community_amd import data as rd
from ray_community_amd.data.block import BlockAccessor
from ray_community_amd.data.extensions import ArrowTensorArray, ArrowTensorType, TensorArray, TensorDtype


def test_arrow_tensor_array_roundtrip_slices_and_ipc():
    x = np.random.default_rng(0).standard_normal((7, 3, 4)).astype(np.float32)
    a = ArrowTensorArray.from_numpy(x)
    assert isinstance(a.type, ArrowTensorType) and a.type.shape == (3, 4)
    assert np.array_equal(a.to_numpy(), x)
    assert np.array_equal(a.slice(2, 3).to_numpy(), x[2:5])  # offsets honoured
    t = pa.table({"t": a, "i": np.arange(7)})
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, t.schema) as w:
        w.write_table(t)
    back = pa.ipc.open_stream(sink.getvalue()).read_all()
    assert back.schema.field("t").type == a.type
    assert np.array_equal(BlockAccessor(back).to_numpy()["t"], x)
    chunked = pa.concat_tables([t.slice(0, 3), t.slice(3)])
    assert np.array_equal(BlockAccessor(chunked).to_numpy()["t"], x)  # multi-chunk column
    for dt in (np.uint8, np.int64, np.bool_):
        y = (np.arange(24).reshape(2, 3, 4) % 2).astype(dt)
        assert np.array_equal(ArrowTensorArray.from_numpy(y).to_numpy(), y)


def test_pandas_tensor_array_behaves_like_a_column():
    x = np.arange(5 * 2 * 2).reshape(5, 2, 2)
    df = pd.DataFrame({"t": TensorArray(x), "k": np.arange(5)})
    assert isinstance(df["t"].dtype, TensorDtype) and df["t"].dtype.shape == (2, 2)
    assert np.array_equal(df["t"][3], x[3])
    assert df[df["k"] % 2 == 0]["t"].array.to_numpy().shape == (3, 2, 2)
    assert np.array_equal(pd.concat([df, df])["t"].array.to_numpy(), np.concatenate([x, x]))
    assert np.array_equal(df.take([4, 0])["t"].array.to_numpy(), x[[4, 0]])
    t = pa.Table.from_pandas(df, preserve_index=False)
    assert isinstance(t.schema.field("t").type, ArrowTensorType)
    assert np.array_equal(t.to_pandas()["t"].array.to_numpy(), x)
    assert TensorDtype.construct_from_string(df["t"].dtype.name) == df["t"].dtype


def test_dataset_tensor_columns_through_parquet_and_batch_formats(shutdown_only, tmp_path):
    ray.init(num_cpus=2)
    imgs = np.random.default_rng(1).integers(0, 255, (24, 8, 8, 3), dtype=np.uint8)
    ds = rd.from_numpy(imgs).map_batches(lambda b: {"img": b["data"], "mean": b["data"].mean(axis=(1, 2, 3))})
    got = np.concatenate([b["img"] for b in ds.iter_batches(batch_size=10, batch_format="numpy")])
    assert got.shape == (24, 8, 8, 3) and np.array_equal(got, imgs)
    # pandas batches: the tensor column is a TensorArray, and a pandas UDF can return one
    def flip(df):
        assert isinstance(df["img"].dtype, TensorDtype)
        df["img"] = TensorArray(df["img"].array.to_numpy()[:, ::-1].copy())
        return df

    flipped = np.concatenate([b["img"] for b in ds.map_batches(flip, batch_format="pandas").iter_batches(
        batch_size=None, batch_format="numpy")])
    assert np.array_equal(flipped, imgs[:, ::-1])
    # arrow batches carry the extension type
    ab = next(iter(ds.iter_batches(batch_size=5, batch_format="pyarrow")))
    assert isinstance(ab.schema.field("img").type, ArrowTensorType)
    # Parquet round trip keeps the row shape
    out = tmp_path / "pq"
    ds.write_parquet(str(out))
    f = sorted(out.glob("*.parquet"))[0]
    assert isinstance(pq.read_table(f).schema.field("img").type, ArrowTensorType)
    back = rd.read_parquet(str(out))
    rows = back.take_all()
    assert len(rows) == 24 and rows[0]["img"].shape == (8, 8, 3)
    stacked = np.stack(sorted((r["img"] for r in rows), key=lambda a: a.tobytes()))
    assert np.array_equal(stacked, np.stack(sorted(imgs, key=lambda a: a.tobytes())))
    assert back.to_pandas()["img"].array.to_numpy().shape == (24, 8, 8, 3)


def test_range_tensor_schema_and_rows(shutdown_only):
    ray.init(num_cpus=2)
    ds = rd.range_tensor(6, shape=(2, 3))
    rows = ds.take(2)
    assert rows[1]["data"].shape == (2, 3)
    tbl = BlockAccessor({"data": np.stack([r["data"] for r in ds.take_all()])}).to_arrow()
    assert tbl.schema.field("data").type.shape == (2, 3)
    with pytest.raises(ValueError):
        ArrowTensorArray.from_numpy(np.float32(1.0))
