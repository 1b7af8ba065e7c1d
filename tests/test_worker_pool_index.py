"""Native worker-pool index (``_native/worker_pool.cpp``): idle stacks per (node, env key), starting
counts and idle reaping the head's dispatch path uses; plus an end-to-end reuse check through the
runtime."""
import ray_community_amd as ray
from ray_community_amd._private.object_store import native


def test_worker_pool_idle_stacks_and_starting():
    p = native().WorkerPool()
    w1, w2, w3 = b"\x01" * 16, b"\x02" * 16, b"\x03" * 16
    assert p.pop_idle("n1", "k") is None
    assert p.add_starting("n1", "k", 1) == 1 and p.add_starting("n1", "k", 1) == 2
    assert p.add_starting("n1", "k", -5) == 0          # never below zero
    assert p.starting("n1", "other") == 0
    p.push_idle("n1", "k", w1, 1.0)
    p.push_idle("n1", "k", w2, 2.0)
    p.push_idle("n1", "gpu", w3, 3.0)
    assert len(p) == 3 and p.idle_count("n1") == 3 and p.is_idle(w1)
    assert p.pop_idle("n1", "k") == w2                  # LIFO: the warmest worker first
    assert p.pop_idle("n1", "gpu") == w3 and p.pop_idle("n1", "gpu") is None
    assert p.remove(w1) and not p.remove(w1)            # died while idle
    assert p.pop_idle("n1", "k") is None and p.idle_count("n1") == 0
    p.push_idle("n1", "k", w1, 1.0)
    p.push_idle("n1", "k", w1, 5.0)                     # re-push moves, never duplicates
    assert len(p) == 1 and p.idle_count("n1") == 1


def test_worker_pool_reap_oldest_first_above_soft_limit():
    p = native().WorkerPool()
    ids = [bytes([i]) * 16 for i in range(1, 6)]
    for i, w in enumerate(ids):
        p.push_idle("n1", "k" if i % 2 else "j", w, float(i))
    p.push_idle("n2", "k", b"\x09" * 16, 0.0)
    # keep 2 idle on n1; only workers idle > 1.5 s at now=4 qualify (since 0, 1, 2): oldest first
    gone = p.reap("n1", 2, 1.5, 4.0)
    assert gone == ids[:3]
    assert p.idle_count("n1") == 2 and p.idle_count("n2") == 1
    assert p.reap("n1", 2, 0.0, 100.0) == []            # at the soft limit: nothing more
    assert p.stats() == {"n1": {"idle": 2, "starting": 0}, "n2": {"idle": 1, "starting": 0}}
    p.add_starting("n2", "k", 2)
    assert sorted(p.drop_node("n2")) == [b"\x09" * 16]
    assert p.starting("n2", "k") == 0 and "n2" not in p.stats()


def test_head_reuses_pooled_workers():
    ray.init(num_cpus=2)
    try:
        @ray.remote
        def pid():
            import os

            return os.getpid()

        first = {ray.get(pid.remote()) for _ in range(6)}
        again = {ray.get(pid.remote()) for _ in range(6)}
        assert again <= first and len(first) <= 2       # sequential calls reuse the pooled workers
        from ray_community_amd._private.worker import _state

        head = _state.get("head")
        if head is not None:
            # no process was spawned beyond the two CPU slots (leased workers are not idle, so only
            # idle + starting + leased together are bounded)
            assert len(head.workers) <= 2 and isinstance(head.wpool.stats(), dict)
    finally:
        ray.shutdown()
