"""Scheduling / placement-group tests (reference: test_placement_group*.py, test_scheduling*.py)."""
import time

import pytest

import ray_community_amd as ray
from ray_community_amd import exceptions as exc
from ray_community_amd.util import placement_group, placement_group_table, remove_placement_group
from ray_community_amd.util.scheduling_strategies import (NodeAffinitySchedulingStrategy,
                                                          PlacementGroupSchedulingStrategy)


def _node_of():
    return ray.get_runtime_context().get_node_id()


def test_multi_node_spread(ray_start_cluster):
    c = ray_start_cluster
    c.add_node(num_cpus=2)
    for _ in range(3):
        c.add_node(num_cpus=2)
    assert len(ray.nodes()) == 4

    @ray.remote(num_cpus=1, scheduling_strategy="SPREAD")
    def where():
        time.sleep(0.2)
        return _node_of()

    nodes = set(ray.get([where.remote() for _ in range(8)]))
    assert len(nodes) == 4


def test_node_affinity(ray_start_cluster):
    c = ray_start_cluster
    c.add_node(num_cpus=1)
    n2 = c.add_node(num_cpus=1, resources={"x": 1})

    @ray.remote
    def where():
        return _node_of()

    s = NodeAffinitySchedulingStrategy(n2.node_id, soft=False)
    assert ray.get(where.options(scheduling_strategy=s).remote()) == n2.node_id

    @ray.remote(resources={"x": 1})
    def on_x():
        return _node_of()

    assert ray.get(on_x.remote()) == n2.node_id


def test_placement_group_strict_spread(ray_start_cluster):
    c = ray_start_cluster
    c.add_node(num_cpus=2)
    c.add_node(num_cpus=2)
    c.add_node(num_cpus=2)
    pg = placement_group([{"CPU": 1}] * 3, strategy="STRICT_SPREAD")
    assert ray.get(pg.ready(), timeout=10)
    t = placement_group_table(pg)
    assert len(set(t["bundles_to_node_id"].values())) == 3

    @ray.remote(num_cpus=1)
    def where():
        return _node_of()

    nodes = ray.get([where.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg, i)).remote()
                     for i in range(3)])
    assert [t["bundles_to_node_id"][i] for i in range(3)] == nodes
    remove_placement_group(pg)
    assert placement_group_table(pg)["state"] == "REMOVED"


def test_placement_group_pack_and_pending(ray_start_regular):
    pg = placement_group([{"CPU": 2}, {"CPU": 2}], strategy="PACK")
    assert pg.wait(10)
    pg2 = placement_group([{"CPU": 2}], strategy="PACK")
    assert not pg2.wait(0.5)  # all 4 CPUs reserved by pg
    remove_placement_group(pg)
    assert pg2.wait(10)

    @ray.remote(num_cpus=1)
    class A:
        def ok(self):
            return 1

    a = A.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg2, 0)).remote()
    assert ray.get(a.ok.remote()) == 1
    remove_placement_group(pg2)
    with pytest.raises(exc.RayActorError):
        ray.get(a.ok.remote(), timeout=10)


def test_placement_group_validation(ray_start_regular):
    with pytest.raises(ValueError):
        placement_group([], strategy="PACK")
    with pytest.raises(ValueError):
        placement_group([{"CPU": 1}], strategy="FOO")


def test_resources_accounting(ray_start_regular):
    total = ray.cluster_resources()["CPU"]

    @ray.remote(num_cpus=2)
    class Holder:
        def ping(self):
            return 1

    h = Holder.remote()
    ray.get(h.ping.remote())
    avail = ray.available_resources().get("CPU", 0)
    assert avail == total - 2
    ray.kill(h)
    deadline = time.time() + 10
    while time.time() < deadline and ray.available_resources().get("CPU", 0) != total:
        time.sleep(0.05)
    assert ray.available_resources()["CPU"] == total


def test_remove_node_fails_tasks(ray_start_cluster):
    c = ray_start_cluster
    c.add_node(num_cpus=1)
    n = c.add_node(num_cpus=1, resources={"only_here": 1})

    @ray.remote(resources={"only_here": 1}, max_retries=0)
    def hang():
        time.sleep(30)

    r = hang.remote()
    time.sleep(1.0)
    c.remove_node(n)
    with pytest.raises((exc.WorkerCrashedError, exc.RayError)):
        ray.get(r, timeout=20)


def test_label_selector_places_tasks_and_actors_on_matching_nodes(ray_start_cluster):
    """``label_selector`` and ``NodeLabelSchedulingStrategy`` hard constraints: work lands only on
    nodes whose labels match (equality, negation, in(...), Exists); an unmatched selector keeps
    the task pending instead of running it anywhere."""
    from ray_community_amd.util.scheduling_strategies import Exists, In, NodeLabelSchedulingStrategy

    c = ray_start_cluster
    if True:
        n_a = c.add_node(num_cpus=2, labels={"accel": "mi355x", "zone": "a"})
        n_b = c.add_node(num_cpus=2, labels={"accel": "cpu", "zone": "b"})

        @ray.remote(num_cpus=0.5)
        def where():
            return ray.get_runtime_context().get_node_id()

        ids_a = {ray.get(where.options(label_selector={"accel": "mi355x"}).remote()) for _ in range(6)}
        assert ids_a == {n_a.node_id}
        ids_b = {ray.get(where.options(label_selector={"accel": "!mi355x", "zone": "in(b,c)"}).remote())
                 for _ in range(6)}
        assert ids_b == {n_b.node_id}
        ids_s = {ray.get(where.options(scheduling_strategy=NodeLabelSchedulingStrategy(
            hard={"zone": In("a"), "accel": Exists()})).remote()) for _ in range(4)}
        assert ids_s == {n_a.node_id}

        @ray.remote(num_cpus=0.5, label_selector={"zone": "b"})
        class A:
            def node(self):
                return ray.get_runtime_context().get_node_id()

        assert ray.get(A.remote().node.remote()) == n_b.node_id
        assert "__labelsel" not in str(ray.cluster_resources())
        pending = where.options(label_selector={"accel": "tpu"}).remote()
        ready, _ = ray.wait([pending], timeout=1.0)
        assert not ready


def test_init_with_cluster_address_connects_to_the_in_process_cluster():
    """The reference's ``cluster = Cluster(initialize_head=True); ray.init(address=cluster.address)``
    pattern: connecting to the session the cluster already started is not a double init."""
    from ray_community_amd.cluster_utils import Cluster

    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    try:
        c.add_node(num_cpus=1, resources={"side": 1})
        ctx = ray.init(address=c.address)
        assert ctx is not None and ray.cluster_resources().get("side") == 1

        @ray.remote(resources={"side": 1})
        def f():
            return "side"

        assert ray.get(f.remote()) == "side"
        with pytest.raises(RuntimeError):
            ray.init()  # a different (new local) session is still a double init
    finally:
        ray.shutdown()
        c.shutdown()
