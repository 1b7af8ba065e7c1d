"""Tracing spans across tasks/actors and profile() timeline events (reference:
python/ray/tests/test_tracing.py, test_advanced*.py timeline checks)."""
import json

import ray_community_amd as ray
from ray_community_amd.util import tracing


def test_trace_propagates_through_nested_tasks_and_actors(shutdown_only, tmp_path):
    ray.init(num_cpus=2, _tracing_startup_hook="ray_community_amd.util.tracing:is_tracing_enabled")

    @ray.remote
    def leaf(x):
        with tracing.start_span("leaf-work", {"x": x}):
            return x + 1

    @ray.remote
    def mid(x):
        return ray.get(leaf.remote(x)) * 2

    @ray.remote
    class A:
        def f(self, x):
            return x - 1

    with tracing.start_span("driver-root") as root:
        assert ray.get(mid.remote(1)) == 4
        a = A.remote()
        assert ray.get(a.f.remote(5)) == 4
    spans = tracing.get_spans(root["trace_id"])
    by_name = {s["name"]: s for s in spans}
    assert {"driver-root", "task::mid", "task::leaf", "leaf-work", "actor_method::A.f"} <= set(by_name), by_name.keys()
    assert by_name["task::mid"]["parent_id"] == root["span_id"]
    assert by_name["task::leaf"]["parent_id"] == by_name["task::mid"]["span_id"]
    assert by_name["leaf-work"]["parent_id"] == by_name["task::leaf"]["span_id"]
    assert by_name["leaf-work"]["attributes"]["x"] == 1
    assert by_name["actor_method::A.f"]["parent_id"] == root["span_id"]
    for s in spans:
        assert s["end"] >= s["start"]
    n = tracing.export_spans(str(tmp_path / "spans.jsonl"), root["trace_id"])
    assert n == len(spans) and len((tmp_path / "spans.jsonl").read_text().splitlines()) == n


def test_failed_task_span_marked_error(shutdown_only):
    ray.init(num_cpus=1)
    tracing.enable_tracing(True)

    @ray.remote(max_retries=0)
    def boom():
        raise ValueError("x")

    ref = boom.remote()
    try:
        ray.get(ref)
    except Exception:
        pass
    spans = [s for s in tracing.get_spans() if s["name"] == "task::boom"]
    assert spans and spans[-1]["status"] == "error"


def test_untraced_by_default_and_profile_events_in_timeline(shutdown_only, tmp_path):
    from ray_community_amd._private.profiling import profile

    ray.init(num_cpus=1)

    @ray.remote
    def work():
        with profile("custom-event", {"k": "v"}):
            return 1

    assert ray.get(work.remote()) == 1
    assert not any(s["name"].startswith("task::") for s in tracing.get_spans())
    path = tmp_path / "tl.json"
    ray.timeline(str(path))
    evs = json.loads(path.read_text())
    custom = [e for e in evs if e["name"] == "custom-event"]
    assert custom and custom[0]["cat"] == "profile" and custom[0]["args"]["k"] == "v"
    assert any(e.get("cat") == "task" for e in evs)
