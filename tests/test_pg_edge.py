"""Placement-group scheduling edge cases (reference test models: python/ray/tests/
test_placement_group*.py (tasks confined to a bundle's resources, bundle_index pinning, removal
frees the reservation, named lookup))."""
import time

import pytest

import ray_community_amd as ray
from ray_community_amd.util.placement_group import (get_placement_group, placement_group,
                                                    remove_placement_group)
from ray_community_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_bundle_capacity_serializes_tasks(session):
    pg = placement_group([{"CPU": 1}], name="edge_one")
    assert pg.wait(10)
    assert get_placement_group("edge_one").id == pg.id

    @ray.remote(num_cpus=1)
    def hold(t):
        time.sleep(t)
        return time.time()

    strat = PlacementGroupSchedulingStrategy(placement_group=pg, placement_group_bundle_index=0)
    t0 = time.time()
    ends = ray.get([hold.options(scheduling_strategy=strat).remote(0.6) for _ in range(3)])
    # one CPU in the bundle: the three tasks ran one after another
    assert max(ends) - t0 >= 1.6
    remove_placement_group(pg)
    deadline = time.time() + 10
    while time.time() < deadline and ray.available_resources().get("CPU", 0) < 4:
        time.sleep(0.1)
    assert ray.available_resources().get("CPU", 0) == 4     # the reservation is released


def test_actor_in_pg_sees_its_group(session):
    pg = placement_group([{"CPU": 1}, {"CPU": 1}], strategy="PACK")
    assert pg.wait(10)

    @ray.remote(num_cpus=1)
    class Where:
        def pg_id(self):
            return ray.get_runtime_context().get_placement_group_id()

    a = Where.options(scheduling_strategy=PlacementGroupSchedulingStrategy(
        placement_group=pg, placement_group_bundle_index=1)).remote()
    assert ray.get(a.pg_id.remote()) == pg.id.hex()
    ray.kill(a)
    remove_placement_group(pg)
