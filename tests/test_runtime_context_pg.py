"""Runtime context inside tasks/actors: placement-group membership and child-task capture,
runtime env, current_actor (reference: python/ray/tests/test_runtime_context.py,
test_placement_group_3.py::test_capture_child_tasks)."""
import pytest

import ray_community_amd as ray
from ray_community_amd.util.placement_group import get_current_placement_group, placement_group
from ray_community_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy


@ray.remote
def _child():
    pg = get_current_placement_group()
    return pg.id.hex() if pg is not None else None


@ray.remote
def _parent():
    ctx = ray.get_runtime_context()
    return (ctx.get_placement_group_id(), ctx.should_capture_child_tasks_in_placement_group(),
            ray.get(_child.remote()))


def test_placement_group_membership_and_capture(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    pg = placement_group([{"CPU": 2}])
    ray.get(pg.ready())
    assert get_current_placement_group() is None  # the driver belongs to no group
    pid, cap, child = ray.get(_parent.options(
        scheduling_strategy=PlacementGroupSchedulingStrategy(pg, placement_group_capture_child_tasks=True)).remote())
    assert pid == pg.id.hex() and cap is True and child == pg.id.hex()
    pid, cap, child = ray.get(_parent.options(
        scheduling_strategy=PlacementGroupSchedulingStrategy(pg)).remote())
    assert pid == pg.id.hex() and cap is False and child is None  # not captured: child runs outside
    assert ray.get(_parent.remote())[0] is None


def test_runtime_env_and_current_actor(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)

    @ray.remote(runtime_env={"env_vars": {"RCA_T_X": "7"}})
    def env():
        import os

        ctx = ray.get_runtime_context()
        return ctx.runtime_env.get("env_vars"), os.environ.get("RCA_T_X"), ctx.get_runtime_env_string()

    ev, val, s = ray.get(env.remote())
    assert ev == {"RCA_T_X": "7"} and val == "7" and "RCA_T_X" in s

    @ray.remote
    class Me:
        def who(self):
            return ray.get_runtime_context().current_actor

        def ping(self):
            return "pong"

    a = Me.remote()
    h = ray.get(a.who.remote())
    assert ray.get(h.ping.remote()) == "pong"
    with pytest.raises(RuntimeError):
        ray.get_runtime_context().current_actor
