"""Ray Data tests (modelled on reference data/tests/test_map.py, test_consumption.py, test_sort.py,
test_all_to_all.py, test_preprocessors)."""
import os

import numpy as np
import pandas as pd
import pytest

import ray_community_amd as ray
from ray_community_amd import data as rd


def test_range_count_take(ray_start_regular):
    ds = rd.range(1000)
    assert ds.count() == 1000
    assert [r["id"] for r in ds.take(5)] == [0, 1, 2, 3, 4]
    assert ds.schema().names == ["id"]
    assert ds.sum("id") == sum(range(1000))


def test_map_batches_fusion_and_filter(ray_start_regular):
    ds = (rd.range(500)
          .map_batches(lambda b: {"id": b["id"], "sq": b["id"] ** 2}, batch_size=64)
          .filter(lambda r: r["id"] % 2 == 0)
          .map(lambda r: {"v": r["sq"] + 1}))
    out = [r["v"] for r in ds.iter_rows()]
    assert out == [i * i + 1 for i in range(0, 500, 2)]


def test_iter_batches_exact_sizes(ray_start_regular):
    ds = rd.range(1003, override_num_blocks=7)
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=100)]
    assert sizes == [100] * 10 + [3]
    assert sum(len(b["id"]) for b in ds.iter_batches(batch_size=100, drop_last=True)) == 1000
    dfs = list(ds.iter_batches(batch_size=500, batch_format="pandas"))
    assert isinstance(dfs[0], pd.DataFrame)


def test_actor_pool_map_batches(ray_start_regular):
    class AddK:
        def __init__(self, k):
            self.k = k

        def __call__(self, b):
            return {"id": b["id"] + self.k}

    ds = rd.range(200).map_batches(AddK, fn_constructor_args=(10,), concurrency=2, batch_size=32)
    assert sorted(r["id"] for r in ds.iter_rows()) == list(range(10, 210))


def test_shuffle_sort_repartition(ray_start_regular):
    ds = rd.range(300, override_num_blocks=5)
    sh = ds.random_shuffle(seed=1)
    vals = [r["id"] for r in sh.iter_rows()]
    assert sorted(vals) == list(range(300)) and vals != list(range(300))
    srt = sh.sort("id", descending=True)
    assert [r["id"] for r in srt.iter_rows()] == list(range(299, -1, -1))
    rp = ds.repartition(3)
    assert rp.num_blocks() == 3 and [r["id"] for r in rp.iter_rows()] == list(range(300))


def test_groupby_aggregate(ray_start_regular):
    items = [{"k": i % 3, "v": float(i)} for i in range(30)]
    ds = rd.from_items(items)
    out = ds.groupby("k").sum("v").take_all()
    assert [(r["k"], r["sum(v)"]) for r in out] == [(0, 135.0), (1, 145.0), (2, 155.0)]
    cnt = ds.groupby("k").count().take_all()
    assert [r["count()"] for r in cnt] == [10, 10, 10]
    mg = ds.groupby("k").map_groups(lambda g: {"k": g["k"][:1], "n": np.array([len(g["v"])])}).take_all()
    assert sorted((r["k"], r["n"]) for r in mg) == [(0, 10), (1, 10), (2, 10)]
    assert ds.mean("v") == pytest.approx(14.5)
    assert ds.max("v") == 29.0


def test_union_zip_limit_split(ray_start_regular):
    a = rd.range(10)
    b = rd.range(5)
    assert a.union(b).count() == 15
    z = rd.range(8).zip(rd.from_items([{"w": i * 10} for i in range(8)]))
    assert [(r["id"], r["w"]) for r in z.iter_rows()] == [(i, i * 10) for i in range(8)]
    assert rd.range(100).limit(7).count() == 7
    parts = rd.range(10).split(3)
    assert [p.count() for p in parts] == [4, 3, 3]
    tr, te = rd.range(100).train_test_split(0.2)
    assert tr.count() == 80 and te.count() == 20


def test_read_write_parquet_csv_json_numpy(ray_start_regular, tmp_path):
    ds = rd.from_items([{"a": i, "b": str(i)} for i in range(20)])
    ds.write_parquet(str(tmp_path / "pq"))
    assert rd.read_parquet(str(tmp_path / "pq")).count() == 20
    ds.write_csv(str(tmp_path / "csv"))
    r = rd.read_csv(str(tmp_path / "csv"))
    assert sorted(x["a"] for x in r.iter_rows()) == list(range(20))
    ds.write_json(str(tmp_path / "js"))
    assert rd.read_json(str(tmp_path / "js")).count() == 20
    arr = np.arange(12).reshape(4, 3)
    rd.from_numpy(arr).write_numpy(str(tmp_path / "np"), column="data")
    back = rd.read_numpy(str(tmp_path / "np")).take_batch(10)["data"]
    assert np.array_equal(back, arr)
    (tmp_path / "t.txt").write_text("hello\nworld\n")
    assert [r["text"] for r in rd.read_text(str(tmp_path / "t.txt")).iter_rows()] == ["hello", "world"]


def test_tensor_blocks_and_torch_batches(ray_start_regular):
    imgs = np.random.randint(0, 255, (16, 8, 8, 3), dtype=np.uint8)
    ds = rd.from_numpy(imgs)
    b = next(iter(ds.iter_torch_batches(batch_size=8, device="cpu")))
    assert tuple(b["data"].shape) == (8, 8, 8, 3)
    from ray_community_amd.data.gpu import ImageNormalize

    out = ds.map_batches(ImageNormalize, fn_constructor_kwargs={"column": "data", "dtype": "float32"},
                         concurrency=1, batch_size=8, batch_format="numpy").take_batch(16)
    assert out["data"].shape == (16, 3, 8, 8)
    ref = (imgs[0].astype(np.float32) / 255 - np.array([0.485, 0.456, 0.406])) / np.array([0.229, 0.224, 0.225])
    assert np.allclose(out["data"][0], ref.transpose(2, 0, 1), atol=1e-4)


def test_preprocessors(ray_start_regular):
    from ray_community_amd.data.preprocessors import (Chain, Concatenator, LabelEncoder, MinMaxScaler,
                                                      OneHotEncoder, StandardScaler)

    ds = rd.from_pandas(pd.DataFrame({"x": [1.0, 2.0, 3.0, 4.0], "y": ["a", "b", "a", "c"], "z": [0, 1, 2, 3]}))
    s = StandardScaler(["x"]).fit(ds)
    out = s.transform(ds).to_pandas()
    assert abs(out["x"].mean()) < 1e-9
    mm = MinMaxScaler(["z"]).fit_transform(ds).to_pandas()
    assert mm["z"].tolist() == [0.0, 1 / 3, 2 / 3, 1.0]
    le = LabelEncoder("y").fit(ds)
    assert le.transform(ds).to_pandas()["y"].tolist() == [0, 1, 0, 2]
    oh = OneHotEncoder(["y"]).fit_transform(ds).to_pandas()
    assert oh["y_a"].tolist() == [1, 0, 1, 0]
    ch = Chain(StandardScaler(["x"]), Concatenator(output_column_name="f", include=["x", "z"]))
    f = ch.fit_transform(ds).take_batch(4)["f"]
    assert f.shape == (4, 2)


def test_train_with_dataset_shards(ray_start_regular, tmp_path):
    from ray_community_amd import train
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.torch import TorchTrainer

    def loop():
        shard = train.get_dataset_shard("train")
        n = sum(len(b["id"]) for b in shard.iter_batches(batch_size=16))
        train.report({"rows": n})

    r = TorchTrainer(loop, datasets={"train": rd.range(100)}, scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(storage_path=str(tmp_path))).fit()
    assert r.metrics["rows"] == 50
