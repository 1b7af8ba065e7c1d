"""Native actor directory (_native/actor_table.cpp): name reservation, node / placement-group /
handle-holder indexes and state counts, and the head using it (named actors, PG removal killing
its actors, a dying handle holder)."""
import pytest

from ray_community_amd._native import _rca_native as native


def test_directory_indexes():
    d = native.ActorDirectory("DEAD")
    d.add(b"a1", "svc", "ns", "drv", b"pg1", "PENDING_CREATION", "C", False)
    d.add(b"a2", None, "ns", b"w1", None, "PENDING_CREATION")
    assert len(d) == 2 and b"a1" in d and b"zz" not in d
    assert d.by_name("ns", "svc") == b"a1" and d.by_name("other", "svc") is None
    assert not d.name_available("ns", "svc") and d.name_available("other", "svc")
    with pytest.raises(ValueError, match="already taken"):
        d.add(b"a3", "svc", "ns", None, None, "PENDING_CREATION")
    d.set_state(b"a1", "ALIVE")
    d.set_node(b"a1", "n1")
    d.set_node(b"a2", "n1")
    assert sorted(d.on_node("n1")) == [b"a1", b"a2"]
    d.set_node(b"a2", "n2")
    assert d.on_node("n1") == [b"a1"] and d.on_node("n2") == [b"a2"]
    assert d.in_pg(b"pg1") == [b"a1"] and d.in_pg(b"pg2") == []
    assert d.state_counts() == {"ALIVE": 1, "PENDING_CREATION": 1}
    # str and bytes holders are distinct keys
    assert d.add_handle(b"a2", "w1") == 2 and d.num_handles(b"a2") == 2
    assert d.drop_holder(b"w1") == [b"a2"] and d.num_handles(b"a2") == 1
    assert d.remove_handle(b"a2", "w1") == 0
    assert d.named("ns") == [b"a1"] and d.named(all_namespaces=True) == [b"a1"]
    # a dead holder frees its name
    d.set_state(b"a1", "DEAD")
    assert d.name_available("ns", "svc") and d.named("ns") == []
    d.add(b"a3", "svc", "ns", None, None, "PENDING_CREATION")
    assert d.by_name("ns", "svc") == b"a3"
    d.remove(b"a1")
    assert b"a1" not in d and d.by_name("ns", "svc") == b"a3" and d.in_pg(b"pg1") == []
    assert d.state_counts() == {"PENDING_CREATION": 2}


def test_head_uses_directory(ray_start_regular):
    import ray_community_amd as ray
    from ray_community_amd.util.placement_group import placement_group, remove_placement_group
    from ray_community_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy

    @ray.remote
    class A:
        def ping(self):
            return 1

    a = A.options(name="dir_a", namespace="dns").remote()
    assert ray.get(a.ping.remote()) == 1
    assert ray.get(ray.get_actor("dir_a", namespace="dns").ping.remote()) == 1
    with pytest.raises(ValueError):
        A.options(name="dir_a", namespace="dns").remote()
    pg = placement_group([{"CPU": 1}])
    ray.get(pg.ready())
    b = A.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg)).remote()
    assert ray.get(b.ping.remote()) == 1
    remove_placement_group(pg)
    with pytest.raises(ray.exceptions.RayActorError):
        ray.get(b.ping.remote(), timeout=30)
    ray.kill(a)
    with pytest.raises(ray.exceptions.RayActorError):
        ray.get(a.ping.remote(), timeout=30)
    # the name is free again once its holder is dead
    c = A.options(name="dir_a", namespace="dns").remote()
    assert ray.get(c.ping.remote()) == 1
