"""Dataset lineage serialization, the legacy write_datasource API and DataIterator.schema /
to_torch (reference: python/ray/data/dataset.py serialize_lineage / deserialize_lineage /
has_serializable_lineage / write_datasource, data/iterator.py)."""
import pytest

import ray_community_amd as ray


@pytest.fixture
def ray2(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    yield


def test_lineage_round_trip_and_in_memory_rejection(ray2):
    ds = ray.data.range(100, override_num_blocks=4).map(lambda r: {"id": r["id"] * 3}).filter(lambda r: r["id"] % 2 == 0)
    assert ds.has_serializable_lineage()
    blob = ds.serialize_lineage()
    assert isinstance(blob, bytes)
    back = ray.data.Dataset.deserialize_lineage(blob)
    assert sorted(r["id"] for r in back.take_all()) == sorted(r["id"] for r in ds.take_all())
    mem = ray.data.from_items([{"a": 1}, {"a": 2}])
    assert not mem.has_serializable_lineage()
    with pytest.raises(ValueError):
        mem.serialize_lineage()
    assert not ds.materialize().has_serializable_lineage()


def test_write_datasource_legacy_api(ray2, tmp_path):
    class Collect:
        def write(self, blocks, ctx, prefix=""):
            import json
            import os

            from ray_community_amd.data.block import BlockAccessor

            n = 0
            for b in blocks:
                rows = list(BlockAccessor(b).iter_rows())
                n += len(rows)
                with open(os.path.join(str(tmp_path), f"{prefix}{ctx['task_idx']}.json"), "w") as f:
                    json.dump([int(r["id"]) for r in rows], f)
            return n

        def on_write_complete(self, results):
            (tmp_path / "done").write_text(str(sum(results)))

    ray.data.range(50, override_num_blocks=5).write_datasource(Collect(), prefix="p")
    assert (tmp_path / "done").read_text() == "50"
    assert len(list(tmp_path.glob("p*.json"))) == 5


def test_iterator_schema_to_torch_and_absent_frameworks(ray2):
    ds = ray.data.from_items([{"x": float(i), "y": i % 2} for i in range(10)])
    it = ds.iterator()
    assert "x" in ds.schema().names and it.schema().names == ds.schema().names
    feats, labels = next(iter(it.to_torch(label_column="y", batch_size=4)))
    assert feats.shape == (4, 1) and labels.shape == (4,)
    with pytest.raises(ImportError):
        ds.to_dask()
    with pytest.raises(ImportError):
        ds.to_tf()
    parts = ray.data.range(20).streaming_split(2)
    assert parts[0].schema().names == ["id"]
