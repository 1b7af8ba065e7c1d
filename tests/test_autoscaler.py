"""Autoscaler over virtual nodes (autoscaler/; reference python/ray/autoscaler/,
tests/test_autoscaler*.py, test_resource_demand_scheduler.py)."""
import time

import pytest

import ray_community_amd as ray
from ray_community_amd.autoscaler import StandardAutoscaler, request_resources
from ray_community_amd.util.placement_group import placement_group


CONFIG = {
    "available_node_types": {
        "accel_worker": {"resources": {"CPU": 2, "accel": 1}, "min_workers": 0, "max_workers": 3},
        "cpu_worker": {"resources": {"CPU": 4}, "min_workers": 0, "max_workers": 2},
    },
    "max_workers": 4,
    "idle_timeout_minutes": 0.002,  # 0.12 s
    "upscaling_speed": 4.0,
}


@pytest.fixture
def one_cpu():
    ray.init(num_cpus=1)
    yield
    ray.shutdown()


@ray.remote(resources={"accel": 1}, num_cpus=1)
def on_accel(x):
    return ray.get_runtime_context().get_node_id(), x


def _types(asc):
    return sorted(asc.provider.non_terminated_nodes().values())


def test_scale_up_for_infeasible_tasks_then_idle_scale_down(one_cpu):
    asc = StandardAutoscaler(CONFIG)
    refs = [on_accel.remote(i) for i in range(3)]
    time.sleep(0.3)
    rep = asc.update()
    # three queued {CPU:1, accel:1} shapes: one accel_worker each (accel: 1 per node), none on cpu_worker
    assert [n for n, _ in rep["launched"]] == ["accel_worker"] * 3
    assert asc.summary()["active_nodes"]["accel_worker"] == 3 and "accel_worker: 3" in asc.info_string()
    assert "accel_worker" in asc.all_node_types
    out = ray.get(refs, timeout=120)
    assert sorted(x for _, x in out) == [0, 1, 2]
    assert len({nid for nid, _ in out}) >= 1
    # nothing queued: no further launches; after the idle timeout every node is removed
    assert asc.update()["launched"] == []
    time.sleep(0.3)
    deadline = time.time() + 30
    while _types(asc) and time.time() < deadline:
        asc.update()
        time.sleep(0.15)
    assert _types(asc) == []


def test_request_resources_min_workers_and_limits(one_cpu):
    cfg = dict(CONFIG, available_node_types={
        "accel_worker": dict(CONFIG["available_node_types"]["accel_worker"], min_workers=1),
        "cpu_worker": CONFIG["available_node_types"]["cpu_worker"]})
    asc = StandardAutoscaler(cfg)
    assert [n for n, _ in asc.update()["launched"]] == ["accel_worker"]  # min_workers
    # standing request: 3 x {CPU: 4} -> cpu_worker is the only type that holds one; capped at 2
    request_resources(bundles=[{"CPU": 4}] * 3)
    asc.update()
    assert _types(asc).count("cpu_worker") == 2
    assert ray.cluster_resources()["CPU"] >= 1 + 2 + 8
    # the request keeps them alive while idle
    time.sleep(0.3)
    asc.update()
    assert _types(asc).count("cpu_worker") == 2
    request_resources()  # clear
    time.sleep(0.3)
    for _ in range(3):
        asc.update()
        time.sleep(0.15)
    assert _types(asc) == ["accel_worker"]  # min_workers stays


def test_pending_placement_group_triggers_scale_up(one_cpu):
    asc = StandardAutoscaler(CONFIG)
    pg = placement_group([{"accel": 1}, {"accel": 1}], strategy="SPREAD")
    time.sleep(0.2)
    rep = asc.update()
    assert len(rep["launched"]) == 2
    assert pg.wait(timeout_seconds=60)
