"""Dataset.streaming_split through the split coordinator (reference:
python/ray/data/_internal/iterator/stream_split_iterator.py, operators/output_splitter.py,
python/ray/data/tests/test_streaming_integration.py): lazy, re-executed per epoch, equal splits,
larger-than-store datasets streaming through, Train shards fed by it."""
import threading
import time

import numpy as np
import pytest

import ray_community_amd as ray


def _consume(its, epochs=1, batch_size=64, sleep=0.0):
    """Each iterator consumed by its own thread; returns {(split, epoch): [ids]}."""
    out = {}

    def run(i, e):
        ids = []
        for b in its[i].iter_batches(batch_size=batch_size, batch_format="numpy"):
            ids.extend(b["id"].tolist())
            if sleep:
                time.sleep(sleep)
        out[(i, e)] = ids

    for e in range(epochs):
        th = [threading.Thread(target=run, args=(i, e)) for i in range(len(its))]
        for t in th:
            t.start()
        for t in th:
            t.join(120)
    return out


def test_streaming_split_is_lazy_and_reshuffles_each_epoch(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    ds = ray.data.range(2000, override_num_blocks=20).random_shuffle()
    t0 = time.time()
    its = ds.streaming_split(2)
    assert time.time() - t0 < 1.0  # returns before anything executes
    out = _consume(its, epochs=2)
    e0 = out[(0, 0)] + out[(1, 0)]
    e1 = out[(0, 1)] + out[(1, 1)]
    assert sorted(e0) == list(range(2000)) and sorted(e1) == list(range(2000))
    assert e0 != e1  # re-executed: a fresh shuffle in epoch 2


def test_streaming_split_equal_rows(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    # uneven blocks (a filter drops a different share of every block) and a total not divisible by 3
    ds = ray.data.range(1001, override_num_blocks=13).filter(lambda r: r["id"] % 7 != 3)
    total = ds.count()
    its = ds.streaming_split(3, equal=True)
    out = _consume(its, epochs=2, batch_size=50)
    for e in range(2):
        counts = [len(out[(i, e)]) for i in range(3)]
        assert counts == [total // 3] * 3, counts
        ids = sum((out[(i, e)] for i in range(3)), [])
        assert len(set(ids)) == len(ids)  # no row twice


def test_streaming_split_dynamic_balances_slow_consumer(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    ds = ray.data.range(4000, override_num_blocks=40)
    its = ds.streaming_split(2, equal=False)
    out = {}

    def run(i, sleep):
        ids = []
        for b in its[i].iter_batches(batch_size=100, batch_format="numpy"):
            ids.extend(b["id"].tolist())
            time.sleep(sleep)
        out[i] = ids

    th = [threading.Thread(target=run, args=(0, 0.0)), threading.Thread(target=run, args=(1, 0.05))]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert sorted(out[0] + out[1]) == list(range(4000))
    assert len(out[0]) > len(out[1])  # the fast consumer pulled more blocks


def test_streaming_split_larger_than_object_store(shutdown_only):
    """~3x the object store's capacity streams through two consumers: blocks are produced as the
    consumers pull and freed once consumed (nothing is materialised up front)."""
    store = 96 << 20
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False, object_store_memory=store)
    rows, row_bytes = 36 * 1024, 8 * 1024  # 288 MB of float64 in 4 MB blocks
    ds = ray.data.range_tensor(rows, shape=(row_bytes // 8,), override_num_blocks=72)
    its = ds.streaming_split(2, equal=True)
    seen = {}

    def run(i):
        n = 0
        for b in its[i].iter_batches(batch_size=512, batch_format="numpy"):
            n += len(b["data"])
        seen[i] = n

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert seen == {0: rows // 2, 1: rows // 2}
    head = ray._private.worker._state.get("head") if hasattr(ray._private.worker, "_state") else None
    if head is not None:
        # streaming keeps the working set inside the store: nothing (or next to nothing) spilled
        assert head.spilled_bytes < store, head.spilled_bytes


def test_streaming_split_materialize_and_validation(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    ds = ray.data.range(100, override_num_blocks=4)
    with pytest.raises(ValueError):
        ds.streaming_split(2, locality_hints=["a"])
    its = ds.streaming_split(1)
    m = its[0].materialize()
    assert m.count() == 100


def test_train_shards_come_from_streaming_split(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    from ray_community_amd import train
    from ray_community_amd.train import ScalingConfig
    from ray_community_amd.train.data_parallel_trainer import DataParallelTrainer

    def loop():
        it = train.get_dataset_shard("train")
        epochs = []
        for _ in range(2):
            epochs.append([int(x) for b in it.iter_batches(batch_size=32, batch_format="numpy") for x in b["id"]])
        train.report({"n0": len(epochs[0]), "n1": len(epochs[1]), "kind": type(it).__name__,
                      "differ": epochs[0] != epochs[1]})

    ds = ray.data.range(600, override_num_blocks=12).random_shuffle()
    res = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                              datasets={"train": ds}).fit()
    assert res.error is None, res.error
    assert res.metrics["n0"] == 300 and res.metrics["n1"] == 300
    assert res.metrics["kind"] == "StreamSplitDataIterator"
    assert res.metrics["differ"]


def test_streaming_split_prefetched_calls_keep_their_order(shutdown_only):
    """One block split equally between two consumers: each consumer's prefetched get() calls run
    concurrently in the coordinator but are answered in call order, so no slice is dropped by a
    later call overtaking an earlier one."""
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    for _ in range(3):
        its = ray.data.range(400, override_num_blocks=1).streaming_split(2, equal=True)
        out = {}

        def run(i):
            out[i] = sorted(r["id"] for r in its[i].materialize().take_all())

        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert len(out[0]) == len(out[1]) == 200
        assert sorted(out[0] + out[1]) == list(range(400))
