"""Native object reference table (``_native/ref_table.cpp``) behind the head's reference counting.

Reference model: src/ray/core_worker/reference_count.h (an object is deleted when its last
reference goes away) and the object directory's node locations. Unit semantics + the property the
head relies on: dropping a dead process's holder key touches only the objects it held.
"""
import time

from ray_community_amd._private.object_store import native


def _oid(i: int) -> bytes:
    return i.to_bytes(4, "little") * 5


def test_holders_pins_and_unreferenced_transitions():
    t = native().RefTable()
    o = _oid(1)
    assert t.add(o) and not t.add(o)
    assert t.unreferenced(o) and not t.referenced(o)
    assert t.add_holder(o, "driver") and not t.add_holder(o, "driver")
    assert t.add_holder(o, "w:aa")
    assert t.num_holders(o) == 2 and sorted(t.holders(o)) == ["driver", "w:aa"]
    assert t.has_holder(o, "w:aa") and not t.has_holder(o, "w:bb")
    assert not t.remove_holder(o, "driver")  # still held by w:aa
    assert not t.pin(o, 2)
    assert not t.remove_holder(o, "w:aa")  # pinned
    assert t.pins(o) == 2 and t.referenced(o)
    assert not t.pin(o, -1)
    assert t.pin(o, -1)  # last pin gone, no holders: unreferenced now
    assert not t.remove_holder(o, "never-seen") or t.unreferenced(o)
    t.erase(o)
    assert not t.contains(o) and len(t) == 0
    assert not t.pin(o, 1) and t.pins(o) == 1  # a pin creates the record


def test_drop_holder_returns_exactly_the_objects_it_kept_alive():
    t = native().RefTable()
    for i in range(10):
        t.add_holder(_oid(i), "w:dead")
    t.add_holder(_oid(3), "driver")  # shared: survives
    t.pin(_oid(5), 1)                # pinned: survives
    t.add_holder(_oid(42), "driver")  # never held by the dead worker
    freed = sorted(t.drop_holder("w:dead"))
    assert freed == sorted(_oid(i) for i in range(10) if i not in (3, 5))
    assert t.held_by("w:dead") == [] and t.drop_holder("w:dead") == []
    assert t.num_holders(_oid(3)) == 1 and t.referenced(_oid(5))
    assert t.stats()["objects"] == 11


def test_clear_refs_and_node_index():
    t = native().RefTable()
    a, b, c = _oid(1), _oid(2), _oid(3)
    for o in (a, b, c):
        t.add_holder(o, "driver")
    t.set_node(a, "n1")
    t.set_node(b, "n1")
    t.set_node(c, "n2")
    assert sorted(t.objects_on_node("n1")) == sorted([a, b]) and t.node(c) == "n2"
    t.set_node(b, "n2")  # moved
    assert t.objects_on_node("n1") == [a] and sorted(t.objects_on_node("n2")) == sorted([b, c])
    t.clear_refs(a)
    assert t.unreferenced(a) and t.held_by("driver") and a not in t.held_by("driver")
    t.erase(c)
    assert t.objects_on_node("n2") == [b] and t.node(c) is None
    t.set_node(b, "")
    assert t.objects_on_node("n2") == [] and t.node(b) is None


def test_drop_holder_cost_scales_with_held_objects_not_table_size():
    t = native().RefTable()
    n = 200_000
    for i in range(n):
        t.add_holder(_oid(i), "driver")
    for i in range(50):
        t.add_holder(_oid(n + i), "w:small")
    t0 = time.perf_counter()
    freed = t.drop_holder("w:small")
    dt = time.perf_counter() - t0
    assert len(freed) == 50
    assert dt < 0.01, dt  # O(held), not O(200k)


def test_head_table_tracks_driver_refs(ray_start_regular):
    """End to end: the in-process head registers the driver as holder of its puts and drops the
    objects from the native table once the driver's refs go out of scope."""
    import gc

    import ray_community_amd as ray
    from ray_community_amd._private.worker import _head

    head = _head()
    refs = [ray.put(bytes(200_000)) for _ in range(20)]  # shm-sized values: head-tracked
    oids = [r.binary() if hasattr(r, "binary") else r.id for r in refs]
    assert all(len(ray.get(r)) == 200_000 for r in refs)
    assert head is not None
    assert all(head.refs.referenced(o) for o in oids)
    del refs
    gc.collect()
    deadline = time.time() + 10
    while time.time() < deadline and any(head.refs.contains(o) for o in oids):
        time.sleep(0.05)
    assert not any(head.refs.contains(o) for o in oids)


def test_kv_table_namespaces_prefixes_and_overwrite():
    """Native internal KV (GCS InternalKV semantics): put reports whether the key was added,
    overwrite=False keeps the old value, None and b"" namespaces are distinct, prefix listing and
    prefix deletion see only matching keys of that namespace."""
    kv = native().KvTable()
    assert kv.put(b"job:1", b"a") and not kv.put(b"job:1", b"b", False)
    assert kv.get(b"job:1") == b"a"
    assert not kv.put("job:1", "c") and kv.get(b"job:1") == b"c"  # str keys are UTF-8 bytes
    kv.put(b"job:2", b"x")
    kv.put(b"jobx", b"y")
    kv.put(b"job:1", b"other", True, b"ns")
    kv.put(b"job:9", b"empty-ns", True, b"")
    assert kv.keys(b"job:") == [b"job:1", b"job:2"]
    assert kv.keys(b"job", b"ns") == [b"job:1"] and kv.keys(b"job", b"") == [b"job:9"]
    assert kv.get(b"job:1", b"ns") == b"other" and kv.get(b"missing") is None
    assert kv.delete(b"job:", None, True) == 2 and kv.keys(b"job") == [b"jobx"]
    assert kv.exists(b"job:1", b"ns") and not kv.exists(b"job:1")
    assert kv.delete(b"job:1", b"ns") == 1 and kv.delete(b"job:1", b"ns") == 0
    assert len(kv) == 2 and kv.nbytes() == len(b"y") + len(b"empty-ns")


def test_internal_kv_through_the_head(ray_start_regular):
    from ray_community_amd.experimental import internal_kv as ikv

    assert not ikv._internal_kv_put(b"k1", b"v1")
    assert ikv._internal_kv_put(b"k1", b"v2")  # existed
    assert ikv._internal_kv_get(b"k1") == b"v2"
    ikv._internal_kv_put("k2", "v", namespace="n")
    assert ikv._internal_kv_list(b"k", namespace="n") == [b"k2"]
    assert ikv._internal_kv_del(b"k", del_by_prefix=True) == 1
    assert not ikv._internal_kv_exists(b"k1")
