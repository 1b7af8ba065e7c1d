"""Streaming union / zip (reference: python/ray/data/_internal/execution/operators/
union_operator.py, zip_operator.py; tests python/ray/data/tests/test_union.py, test_zip.py).
Here both are streaming operators: the other datasets execute concurrently, blocks flow out as
they are ready, and zip aligns rows across differently blocked inputs without materialising
either side."""
import time

import numpy as np
import pytest

import ray_community_amd as ray


@pytest.fixture
def ray4(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    yield


def test_zip_aligns_differently_blocked_inputs(ray4):
    a = ray.data.range(1000, override_num_blocks=7)
    b = ray.data.range(1000, override_num_blocks=3).map(lambda r: {"w": r["id"] * 10})
    rows = a.zip(b).take_all()
    assert len(rows) == 1000
    assert all(r["w"] == 10 * r["id"] for r in rows)
    assert [r["id"] for r in rows] == list(range(1000))
    # column name clash: the right side's column gets a suffix
    z = ray.data.range(10).zip(ray.data.range(10, override_num_blocks=4)).take_all()
    assert z[3] == {"id": 3, "id_1": 3}


def test_zip_row_count_mismatch_raises(ray4):
    with pytest.raises(Exception, match="different number of rows"):
        ray.data.range(10).zip(ray.data.range(11)).take_all()


def test_union_ordered_and_unordered(ray4):
    a, b, c = ray.data.range(30, override_num_blocks=3), ray.data.range(20, override_num_blocks=4), ray.data.range(5)
    got = [r["id"] for r in a.union(b, c).take_all()]
    assert got == list(range(30)) + list(range(20)) + list(range(5))
    ctx = ray.data.DataContext.get_current()
    prev = ctx.execution_options.preserve_order
    ctx.execution_options.preserve_order = False
    try:
        got = sorted(r["id"] for r in a.union(b).take_all())
        assert got == sorted(list(range(30)) + list(range(20)))
    finally:
        ctx.execution_options.preserve_order = prev
    assert a.union(a).count() == 60


def test_union_streams_without_waiting_for_the_other_input(ray4):
    """The first union output is available long before the slow other input has finished."""

    def slow(batch):
        time.sleep(0.4)
        return batch

    a = ray.data.range(40, override_num_blocks=4)
    b = ray.data.range(200, override_num_blocks=20).map_batches(slow, batch_size=None)
    t0 = time.time()
    it = iter(a.union(b).iter_batches(batch_size=10, batch_format="numpy"))
    first = next(it)
    t_first = time.time() - t0
    n = len(first["id"]) + sum(len(x["id"]) for x in it)
    t_all = time.time() - t0
    assert n == 240
    assert t_first < t_all / 2, (t_first, t_all)


def test_zip_streams_larger_than_object_store(shutdown_only):
    """Two 192 MB inputs zipped through a 96 MB object store without spilling: only a window of
    blocks of each side (and of zipped output) is alive at a time. (Windows are counted in
    blocks, so the blocks are kept small against the store here, as the reference's 128 MB
    target block size is against a store of 30 % of RAM.)"""
    store = 96 << 20
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False, object_store_memory=store)
    rows, width = 24 * 1024, 1024  # 8 KB rows: 192 MB per side
    a = ray.data.range_tensor(rows, shape=(width,), override_num_blocks=192)
    b = ray.data.range_tensor(rows, shape=(width,), override_num_blocks=128)
    n, ok = 0, True
    for batch in a.zip(b).iter_batches(batch_size=1024, batch_format="numpy"):
        n += len(batch["data"])
        ok &= bool(np.array_equal(batch["data"][:, 0], batch["data_1"][:, 0]))
    assert n == rows and ok
    head = ray._private.worker._state.get("head") if hasattr(ray._private.worker, "_state") else None
    if head is not None:
        assert head.spilled_bytes == 0, head.spilled_bytes


def test_union_and_zip_stop_early_without_hanging(ray4):
    """A limit downstream of a streaming union / zip stops the side inputs' executions too."""
    def slow(batch):
        time.sleep(0.05)
        return batch

    a = ray.data.range(1000, override_num_blocks=50).map_batches(slow, batch_size=None)
    b = ray.data.range(1000, override_num_blocks=50).map_batches(slow, batch_size=None)
    t0 = time.time()
    assert len(a.union(b).limit(25).take_all()) == 25
    assert len(a.zip(b.map(lambda r: {"w": r["id"]})).limit(7).take_all()) == 7
    assert time.time() - t0 < 30
    # the session stays usable after the early stops
    assert ray.data.range(10).union(ray.data.range(5)).count() == 15
