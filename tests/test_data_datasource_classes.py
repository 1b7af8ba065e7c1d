"""ray.data.datasource classes (reference: python/ray/data/datasource/__init__.py and
data/tests/test_partitioning.py, test_file_based_datasource.py, test_datasink.py):
FileBasedDatasource subclasses, Partitioning / PathPartitionFilter, the built-in datasources,
FilenameProvider and DummyOutputDatasink."""
import os
import sqlite3

import numpy as np
import pandas as pd
import pytest

import ray_community_amd as ray
from ray_community_amd.data.datasource import (BigQueryDatasource, BinaryDatasource, CSVDatasource,
                                               DummyOutputDatasink, FileBasedDatasource, FileExtensionFilter,
                                               FilenameProvider, JSONDatasource, MongoDatasource,
                                               NumpyDatasource, Partitioning, PartitionStyle, PathPartitionFilter,
                                               PathPartitionParser, RandomIntRowDatasource, RangeDatasource,
                                               SQLDatasource, TextDatasource, TorchDatasource)


class _KVDatasource(FileBasedDatasource):
    """A toy format: one ``key=value`` pair per line."""
    _FILE_EXTENSIONS = ["kv"]

    def _read_stream(self, f, path):
        keys, vals = [], []
        for line in f.read().decode().splitlines():
            k, v = line.split("=", 1)
            keys.append(k)
            vals.append(int(v))
        yield {"key": np.asarray(keys, dtype=object), "value": np.asarray(vals)}


def test_partition_parser_and_filter_units(tmp_path):
    p = PathPartitionParser.of(base_dir="/data")
    assert p("/data/year=2024/month=05/x.parquet") == {"year": "2024", "month": "05"}
    d = PathPartitionParser(Partitioning("dir", base_dir="/data", field_names=["year", "month"],
                                         field_types={"year": int}))
    assert d("/data/2024/05/x.csv") == {"year": 2024, "month": "05"}
    with pytest.raises(ValueError):
        Partitioning(PartitionStyle.DIRECTORY)  # DIRECTORY needs field_names
    f = PathPartitionFilter.of(lambda v: v["year"] == "2024", base_dir="/data")
    assert f(["/data/year=2024/a.csv", "/data/year=2023/b.csv", "/data/c.csv"]) == ["/data/year=2024/a.csv"]
    assert FileExtensionFilter(["csv"], allow_if_no_extension=True)(["a.CSV", "b.json", "c"]) == ["a.CSV", "c"]


def test_file_based_datasource_subclass(ray_start_regular, tmp_path):
    for part in ("a", "b"):
        d = tmp_path / f"group={part}"
        d.mkdir()
        for i in range(3):
            (d / f"f{i}.kv").write_text("\n".join(f"{part}{i}_{j}={10 * i + j}" for j in range(4)))
    (tmp_path / "group=a" / "ignored.txt").write_text("not=1")
    src = _KVDatasource(str(tmp_path), partitioning=Partitioning("hive"), include_paths=True)
    tasks = src.get_read_tasks(2)
    assert len(tasks) == 2 and src.estimate_inmemory_data_size() > 0
    ds = ray.data.read_datasource(src, parallelism=2)
    df = ds.to_pandas()
    assert len(df) == 24 and set(df["group"]) == {"a", "b"}
    assert all(p.endswith(".kv") for p in df["path"])
    assert df["value"].sum() == 2 * sum(10 * i + j for i in range(3) for j in range(4))
    only_b = _KVDatasource(str(tmp_path), partitioning=Partitioning("hive"),
                           partition_filter=PathPartitionFilter.of(lambda v: v["group"] == "b"))
    assert set(ray.data.read_datasource(only_b).to_pandas()["group"]) == {"b"}


def test_directory_partitioning_and_partition_filter_on_readers(ray_start_regular, tmp_path):
    for year in (2023, 2024):
        for month in ("01", "02"):
            d = tmp_path / str(year) / month
            d.mkdir(parents=True)
            pd.DataFrame({"x": [year * 100 + int(month)]}).to_csv(d / "part.csv", index=False)
    ds = ray.data.read_csv(str(tmp_path), partitioning=Partitioning("dir", field_names=["year", "month"],
                                                                      field_types={"year": int}))
    df = ds.to_pandas().sort_values("x")
    assert list(df["year"]) == [2023, 2023, 2024, 2024] and list(df["month"]) == ["01", "02", "01", "02"]
    pf = PathPartitionFilter.of(lambda v: v["month"] == "02", style="dir", field_names=["year", "month"])
    assert sorted(ray.data.read_csv(str(tmp_path), partition_filter=pf).to_pandas()["x"]) == [202302, 202402]

    out = tmp_path / "hive"
    ray.data.from_items([{"k": k, "v": i} for i, k in enumerate("aabbc")]).write_parquet(str(out),
                                                                                       partition_cols=["k"])
    kept = ray.data.read_parquet(str(out), partition_filter=PathPartitionFilter.of(lambda v: v["k"] != "b"))
    assert sorted(kept.to_pandas()["k"]) == ["a", "a", "c"]


def test_builtin_file_datasources(ray_start_regular, tmp_path):
    pd.DataFrame({"a": [1, 2, 3]}).to_csv(tmp_path / "t.csv", index=False)
    pd.DataFrame({"b": [4, 5]}).to_json(tmp_path / "t.json", orient="records", lines=True)
    np.save(tmp_path / "t.npy", np.arange(6).reshape(3, 2))
    (tmp_path / "t.txt").write_text("one\n\ntwo\n")
    (tmp_path / "blob.bin").write_bytes(b"\x00\x01\x02")
    assert ray.data.read_datasource(CSVDatasource(str(tmp_path))).to_pandas()["a"].tolist() == [1, 2, 3]
    assert ray.data.read_datasource(JSONDatasource(str(tmp_path))).to_pandas()["b"].tolist() == [4, 5]
    assert ray.data.read_datasource(NumpyDatasource(str(tmp_path))).count() == 3
    txt = ray.data.read_datasource(TextDatasource(str(tmp_path / "t.txt"))).take_all()
    assert [r["text"] for r in txt] == ["one", "two"]
    blob = ray.data.read_datasource(BinaryDatasource(str(tmp_path / "blob.bin"))).take_all()
    assert blob[0]["bytes"] == b"\x00\x01\x02"


def test_non_file_datasources(ray_start_regular, tmp_path):
    assert ray.data.read_datasource(RangeDatasource(10), parallelism=3).sum("id") == 45
    t = ray.data.read_datasource(RangeDatasource(4, block_format="tensor", tensor_shape=(2,)))
    assert t.take_all()[3]["data"].tolist() == [3, 3]
    r = ray.data.read_datasource(RandomIntRowDatasource(20, 3), parallelism=4)
    assert r.count() == 20 and set(r.columns()) == {"c_0", "c_1", "c_2"}
    items = ray.data.read_datasource(TorchDatasource([(i, i * i) for i in range(5)]), parallelism=2).take_all()
    assert [tuple(x["item"]) for x in items] == [(i, i * i) for i in range(5)]
    db = str(tmp_path / "t.db")
    con = sqlite3.connect(db)
    con.execute("CREATE TABLE t (a INTEGER)")
    con.executemany("INSERT INTO t VALUES (?)", [(i,) for i in range(7)])
    con.commit()
    con.close()
    sql = ray.data.read_datasource(SQLDatasource("SELECT a FROM t", lambda: sqlite3.connect(db)), parallelism=3)
    assert sql.sum("a") == 21
    with pytest.raises(ImportError):
        MongoDatasource(uri="mongodb://x")
    with pytest.raises(ImportError):
        BigQueryDatasource(project_id="p")


def test_filename_provider_and_dummy_sink(ray_start_regular, tmp_path):
    class _Names(FilenameProvider):
        def get_filename_for_block(self, block, task_index, block_index):
            return f"part-{task_index:03d}.csv"

    ray.data.range(30, override_num_blocks=3).write_csv(str(tmp_path / "out"), filename_provider=_Names())
    assert sorted(os.listdir(tmp_path / "out")) == ["part-000.csv", "part-001.csv", "part-002.csv"]
    assert ray.data.read_csv(str(tmp_path / "out")).count() == 30
    sink = DummyOutputDatasink()
    ray.data.range(12, override_num_blocks=4).write_datasink(sink)
    assert sink.rows_written == 12 and sink.num_ok == 1


def test_multi_key_sort_and_boundaries(ray_start_regular):
    rows = [{"a": i % 3, "b": (7 * i) % 5, "c": i} for i in range(30)]
    out = ray.data.from_items(rows, override_num_blocks=4).sort(["a", "b"], descending=[False, True]).take_all()
    assert [(r["a"], r["b"]) for r in out] == sorted([(r["a"], r["b"]) for r in rows], key=lambda t: (t[0], -t[1]))
    ds = ray.data.range(100, override_num_blocks=5).sort("id", boundaries=[25, 50, 75])
    assert ds.num_blocks() == 4 if hasattr(ds, "num_blocks") else True
    assert [r["id"] for r in ds.take_all()] == list(range(100))
    desc = ray.data.range(50, override_num_blocks=3).sort("id", descending=True).take_all()
    assert [r["id"] for r in desc] == list(range(49, -1, -1))
    with pytest.raises(ValueError):
        ray.data.range(3).sort(["id"], descending=[True, False])


def test_execution_resources_arithmetic():
    from ray_community_amd.data import BlockMetadata, ExecutionResources as E

    a, b = E(4, 1, 100), E(2, None, 50)
    assert a.subtract(b) == E(2, 1.0, 50) and a.min(b) == E(2, 1, 50) and a.max(b) == E(4, None, 100)
    assert E.zero().is_zero() and not a.is_zero() and a.copy() == a
    assert not E(1, 0, 0).subtract(E(2, 0, 0)).is_non_negative()
    assert BlockMetadata is not None
