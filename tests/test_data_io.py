"""Data sources and sinks: custom Datasink, SQL (sqlite3), WebDataset tar shards, TFRecords
(tf.train.Example wire format), images, refs constructors, random-access lookups.
Reference tests: python/ray/data/tests/test_sql.py, test_webdataset.py, test_tfrecords.py,
test_image.py, test_random_access.py, test_datasink.py."""
import os
import sqlite3
import struct

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import data as rd
from ray_community_amd.data import datasource as dsrc


@pytest.fixture
def ray2():
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    yield
    ray.shutdown()


class _CollectSink(rd.Datasink):
    def __init__(self, path):
        self.path = path
        self.started = False

    def on_write_start(self):
        self.started = True
        os.makedirs(self.path, exist_ok=True)

    def write(self, blocks, ctx):
        n = 0
        with open(os.path.join(self.path, f"{ctx.task_idx}.txt"), "w") as f:
            for b in blocks:
                for r in rd.BlockAccessor(b).iter_rows():
                    f.write(f"{r['id']}\n")
                    n += 1
        return n

    def on_write_complete(self, results):
        with open(os.path.join(self.path, "_done"), "w") as f:
            f.write(str(sum(results)))


def test_custom_datasink(ray2, tmp_path):
    ds = rd.range(100, override_num_blocks=4)
    sink = _CollectSink(str(tmp_path / "out"))
    ds.write_datasink(sink)
    assert open(tmp_path / "out" / "_done").read() == "100"
    got = sorted(int(x) for f in os.listdir(tmp_path / "out") if f.endswith(".txt")
                 for x in open(tmp_path / "out" / f).read().split())
    assert got == list(range(100))


def test_sql_roundtrip(ray2, tmp_path):
    db = str(tmp_path / "t.db")
    con = sqlite3.connect(db)
    con.execute("CREATE TABLE m (id INTEGER, score REAL, name TEXT)")
    con.commit()
    con.close()
    factory = lambda: sqlite3.connect(db)  # noqa: E731
    rows = [{"id": i, "score": i * 0.5, "name": f"n{i}"} for i in range(50)]
    rd.from_items(rows, override_num_blocks=5).write_sql("INSERT INTO m VALUES (?, ?, ?)", factory)
    back = rd.read_sql("SELECT * FROM m ORDER BY id", factory).take_all()
    assert [r["id"] for r in back] == list(range(50)) and back[3]["name"] == "n3"
    sharded = rd.read_sql("SELECT * FROM m ORDER BY id", factory, override_num_blocks=4)
    assert sharded.num_blocks() == 4 if hasattr(sharded, "num_blocks") else True
    assert sorted(r["id"] for r in sharded.take_all()) == list(range(50))
    assert rd.read_sql("SELECT COUNT(*) AS c FROM m WHERE score > 10", factory).take_all()[0]["c"] == 29


def test_webdataset_roundtrip(ray2, tmp_path):
    rows = [{"__key__": f"s{i:03d}", "cls": i % 3, "json": {"i": i}, "txt": f"caption {i}",
             "png": np.full((4, 5, 3), i, dtype=np.uint8)} for i in range(12)]
    rd.from_items(rows, override_num_blocks=3).write_webdataset(str(tmp_path / "wds"))
    shards = sorted(os.listdir(tmp_path / "wds"))
    assert len(shards) == 3 and all(s.endswith(".tar") for s in shards)
    back = sorted(rd.read_webdataset(str(tmp_path / "wds")).take_all(), key=lambda r: r["__key__"])
    assert [r["cls"] for r in back] == [i % 3 for i in range(12)]
    assert back[5]["json"] == {"i": 5} and back[5]["txt"] == "caption 5"
    assert back[7]["png"].shape == (4, 5, 3) and int(back[7]["png"][0, 0, 0]) == 7
    raw = rd.read_webdataset(str(tmp_path / "wds"), decoder=False, suffixes=["txt"]).take(1)[0]
    assert isinstance(raw["txt"], bytes) and "png" not in raw


def test_tfrecords_roundtrip_and_wire_format(ray2, tmp_path):
    rows = [{"label": i, "weight": float(i) / 4, "name": f"r{i}", "vec": [i, i + 1, i + 2]} for i in range(20)]
    rd.from_items(rows, override_num_blocks=2).write_tfrecords(str(tmp_path / "tfr"))
    files = sorted(os.listdir(tmp_path / "tfr"))
    assert len(files) == 2
    # TFRecord framing: u64 length, masked crc32c of the length, payload, masked crc32c
    raw = open(tmp_path / "tfr" / files[0], "rb").read()
    (n,) = struct.unpack("<Q", raw[:8])
    assert struct.unpack("<I", raw[8:12])[0] == dsrc._masked_crc(raw[:8])
    assert struct.unpack("<I", raw[12 + n: 16 + n])[0] == dsrc._masked_crc(raw[12:12 + n])
    assert dsrc._crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    back = sorted(rd.read_tfrecords(str(tmp_path / "tfr"), verify_checksums=True).take_all(), key=lambda r: r["label"])
    assert [r["label"] for r in back] == list(range(20))
    assert back[3]["name"] == b"r3" and abs(back[3]["weight"] - 0.75) < 1e-6 and list(back[3]["vec"]) == [3, 4, 5]


def test_write_images_and_read_back(ray2, tmp_path):
    imgs = [{"image": np.full((6, 7, 3), 10 * i, dtype=np.uint8)} for i in range(5)]
    rd.from_items(imgs).write_images(str(tmp_path / "img"), column="image")
    files = sorted(os.listdir(tmp_path / "img"))
    assert len(files) == 5 and files[0].endswith(".png")
    back = rd.read_images(str(tmp_path / "img")).take_all()
    assert sorted(int(r["image"][0, 0, 0]) for r in back) == [0, 10, 20, 30, 40]


def test_refs_constructors_and_input_files(ray2, tmp_path):
    import pandas as pd
    import pyarrow as pa

    df_refs = [ray.put(pd.DataFrame({"a": [1, 2]})), ray.put(pd.DataFrame({"a": [3]}))]
    assert sorted(r["a"] for r in rd.from_pandas_refs(df_refs).take_all()) == [1, 2, 3]
    t_ref = ray.put(pa.table({"b": [5, 6]}))
    assert [r["b"] for r in rd.from_arrow_refs(t_ref).take_all()] == [5, 6]
    rd.from_items([{"x": i} for i in range(6)], override_num_blocks=2).write_parquet(str(tmp_path / "pq"))
    ds = rd.read_parquet_bulk(str(tmp_path / "pq"))
    assert len(ds.input_files()) == 2 and all(f.endswith(".parquet") for f in ds.input_files())
    assert ds.copy().count() == 6


def test_random_access_dataset(ray2):
    ds = rd.from_items([{"k": int(k), "v": f"val{k}"} for k in np.random.RandomState(0).permutation(200)],
                       override_num_blocks=8)
    rad = ds.to_random_access_dataset("k", num_workers=3)
    assert ray.get(rad.get_async(17))["v"] == "val17"
    assert ray.get(rad.get_async(1000)) is None and ray.get(rad.get_async(-5)) is None
    got = rad.multiget([5, 199, 0, 300, 42])
    assert [g["v"] if g else None for g in got] == ["val5", "val199", "val0", None, "val42"]
    assert "worker 0" in rad.stats()


def test_hive_partitioned_parquet_and_csv_options(ray_start_regular, tmp_path):
    """write_parquet(partition_cols=...) writes hive directories without the partition columns;
    read_parquet restores them as string columns (reference default Partitioning("hive")) and
    honours columns= / filter=; read_csv forwards pyarrow ParseOptions."""
    import pyarrow.csv as pcsv
    import pyarrow.dataset as pads

    from ray_community_amd import data

    ds = data.from_items([{"k": i % 3, "g": "ab"[i % 2], "v": i} for i in range(30)])
    out = str(tmp_path / "pq")
    ds.write_parquet(out, partition_cols=["k", "g"])
    dirs = sorted(os.listdir(out))
    assert dirs == ["k=0", "k=1", "k=2"] and sorted(os.listdir(os.path.join(out, "k=0"))) == ["g=a", "g=b"]
    back = data.read_parquet(out)
    rows = sorted((r["k"], r["g"], r["v"]) for r in back.take_all())
    assert rows == sorted((str(i % 3), "ab"[i % 2], i) for i in range(30))
    assert data.read_parquet(out, columns=["v", "k"]).columns() == ["v", "k"]
    assert data.read_parquet(out, partitioning=None).columns() == ["v"]
    small = data.read_parquet(out, filter=pads.field("v") < 5)
    assert sorted(r["v"] for r in small.take_all()) == [0, 1, 2, 3, 4]
    tsv = tmp_path / "t.csv"
    tsv.write_text("a\tb\n1\t2\n3\t4\n")
    t = data.read_csv(str(tsv), parse_options=pcsv.ParseOptions(delimiter="\t"))
    assert t.take_all() == [{"a": 1, "b": 2}, {"a": 3, "b": 4}]


def test_min_rows_per_file(ray_start_regular, tmp_path):
    from ray_community_amd import data

    ds = data.range(100, override_num_blocks=10)
    out = str(tmp_path / "csv")
    ds.write_csv(out, min_rows_per_file=30)
    files = os.listdir(out)
    assert len(files) == 3
    assert data.read_csv(out).count() == 100
