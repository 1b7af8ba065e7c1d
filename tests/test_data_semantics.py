"""Data transform semantics against plain-Python expectations (reference: data/tests/
test_all_to_all.py, test_map.py, test_split.py, test_zip.py, test_consumption.py)."""
import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import data as rd


@pytest.fixture(scope="module")
def ray4():
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    yield
    ray.shutdown()


def test_seeded_shuffle_is_reproducible_permutation(ray4):
    a = [r["id"] for r in rd.range(200, override_num_blocks=5).random_shuffle(seed=7).take_all()]
    b = [r["id"] for r in rd.range(200, override_num_blocks=5).random_shuffle(seed=7).take_all()]
    assert a == b and sorted(a) == list(range(200)) and a != list(range(200))


def test_sort_descending_and_multi_block(ray4):
    rows = [{"k": int(x), "v": i} for i, x in enumerate(np.random.RandomState(1).randint(0, 50, 300))]
    out = rd.from_items(rows, override_num_blocks=6).sort("k", descending=True).take_all()
    assert [r["k"] for r in out] == sorted((r["k"] for r in rows), reverse=True)


def test_groupby_map_groups_and_multi_agg(ray4):
    from ray_community_amd.data.aggregate import Count, Max, Mean, Sum

    rows = [{"g": i % 3, "x": float(i)} for i in range(30)]
    ds = rd.from_items(rows, override_num_blocks=4)
    agg = {r["g"]: r for r in ds.groupby("g").aggregate(Count(), Sum("x"), Max("x"), Mean("x")).take_all()}
    for g in range(3):
        xs = [float(i) for i in range(30) if i % 3 == g]
        assert agg[g]["count()"] == len(xs) and agg[g]["sum(x)"] == sum(xs) and agg[g]["max(x)"] == max(xs)
        assert abs(agg[g]["mean(x)"] - sum(xs) / len(xs)) < 1e-9
    norm = ds.groupby("g").map_groups(lambda b: {"g": b["g"], "xc": b["x"] - b["x"].mean()}).take_all()
    assert abs(sum(r["xc"] for r in norm)) < 1e-9 and len(norm) == 30


def test_flat_map_filter_add_drop_select(ray4):
    ds = rd.range(10).flat_map(lambda r: [{"id": r["id"]}, {"id": -r["id"]}])
    assert ds.count() == 20
    ds = ds.filter(lambda r: r["id"] > 0).add_column("sq", lambda b: b["id"] ** 2)
    assert sorted((r["id"], r["sq"]) for r in ds.take_all()) == [(i, i * i) for i in range(1, 10)]
    assert ds.drop_columns(["sq"]).columns() == ["id"] and ds.select_columns(["sq"]).columns() == ["sq"]


def test_splits(ray4):
    ds = rd.range(100, override_num_blocks=7)
    parts = ds.split(3, equal=True)
    sizes = [p.count() for p in parts]
    assert sizes == [33, 33, 33]
    a, b, c = ds.split_at_indices([10, 45])
    assert (a.count(), b.count(), c.count()) == (10, 35, 55)
    assert [r["id"] for r in b.take(2)] == [10, 11]
    tr, te = ds.train_test_split(test_size=0.25)
    assert (tr.count(), te.count()) == (75, 25)
    p = ds.split_proportionately([0.2, 0.3])
    assert [x.count() for x in p] == [20, 30, 50]


def test_zip_union_limit_unique(ray4):
    a = rd.range(6, override_num_blocks=2)
    b = rd.from_items([{"y": i * 10} for i in range(6)], override_num_blocks=3)
    z = a.zip(b).take_all()
    assert [(r["id"], r["y"]) for r in z] == [(i, i * 10) for i in range(6)]
    u = a.union(a)
    assert u.count() == 12 and sorted(u.unique("id")) == list(range(6))
    assert a.limit(4).count() == 4


def test_iter_batches_shapes_and_local_shuffle(ray4):
    ds = rd.range(103, override_num_blocks=4)
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=10, batch_format="numpy")]
    assert sizes == [10] * 10 + [3]
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=10, drop_last=True)]
    assert sizes == [10] * 10
    got = np.concatenate([b["id"] for b in ds.iter_batches(batch_size=16, local_shuffle_buffer_size=32,
                                                           local_shuffle_seed=3)])
    assert sorted(got.tolist()) == list(range(103)) and got.tolist() != list(range(103))
    import torch

    tb = next(iter(ds.iter_torch_batches(batch_size=8, dtypes=torch.float32)))
    assert tb["id"].dtype == torch.float32 and tb["id"].shape == (8,)


def test_map_batches_formats_and_stats(ray4):
    import pandas as pd

    ds = rd.range(20).map_batches(lambda df: df.assign(z=df["id"] * 2), batch_format="pandas", batch_size=5)
    assert sorted(r["z"] for r in ds.take_all()) == [2 * i for i in range(20)]
    ds = rd.range(20).map_batches(lambda b: {"id": b["id"] + 1}, batch_format="numpy")
    assert ds.sum("id") == sum(range(1, 21)) and ds.min("id") == 1 and ds.max("id") == 20
    assert "Dataset" in ds.materialize().stats()
    df = ds.to_pandas()
    assert isinstance(df, pd.DataFrame) and len(df) == 20
