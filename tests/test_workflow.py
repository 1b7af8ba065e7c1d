"""Durable workflows (reference tests: python/ray/workflow/tests/test_basic_workflows*.py,
test_recovery.py, test_dynamic_workflow_ref.py)."""
import os

import pytest

import ray_community_amd as ray
from ray_community_amd import workflow
from ray_community_amd.dag import InputNode


@pytest.fixture
def wf(tmp_path):
    ray.init(num_cpus=4)
    workflow.init(str(tmp_path / "wf_storage"))
    yield tmp_path
    ray.shutdown()


@ray.remote
def add(a, b):
    return a + b


@ray.remote
def double(x):
    return 2 * x


def test_run_and_outputs(wf):
    with InputNode() as inp:
        dag = add.bind(double.bind(inp), 3)
    assert workflow.run(dag, 5, workflow_id="w1", metadata={"k": "v"}) == 13
    assert workflow.get_status("w1") == workflow.WorkflowStatus.SUCCESSFUL
    assert workflow.get_output("w1") == 13
    assert workflow.get_output("w1", task_id="double") == 10
    assert workflow.get_metadata("w1")["user_metadata"] == {"k": "v"}
    assert ("w1", workflow.WorkflowStatus.SUCCESSFUL) in workflow.list_all()
    # running an existing successful workflow returns its stored output
    assert workflow.run(dag, 999, workflow_id="w1") == 13


def test_failure_and_resume_skips_checkpointed_tasks(wf):
    marker = wf / "counter"
    flag = wf / "fail_once"
    flag.write_text("1")

    @ray.remote
    def count(x):
        with open(marker, "a") as f:
            f.write("x")
        return x + 1

    @ray.remote
    def flaky(x):
        if os.path.exists(flag):
            raise ValueError("transient failure")
        return x * 10

    dag = flaky.options(max_retries=0).bind(count.bind(1))
    with pytest.raises(Exception):
        workflow.run(dag, workflow_id="w2")
    assert workflow.get_status("w2") == workflow.WorkflowStatus.FAILED
    os.remove(flag)
    assert workflow.resume("w2") == 20
    assert marker.read_text() == "x"  # count() ran once: its output was checkpointed


@ray.remote
def fact(n, acc=1):
    if n <= 1:
        return acc
    return workflow.continuation(fact.bind(n - 1, acc * n))


def test_continuation_recursion(wf):
    assert workflow.run(fact.bind(6), workflow_id="w3") == 720
    assert workflow.get_output("w3", task_id="fact.fact.fact") is not None


def test_catch_exceptions_and_cancel_delete(wf):
    @ray.remote
    def boom():
        raise RuntimeError("x")

    res, err = workflow.run(workflow.options(catch_exceptions=True)(boom).bind(), workflow_id="w4")
    assert res is None and isinstance(err, Exception)

    @ray.remote
    def slow():
        import time

        time.sleep(2)
        return 1

    ref = workflow.run_async(add.bind(slow.bind(), slow.bind()), workflow_id="w5")
    workflow.cancel("w5")
    with pytest.raises(Exception):
        ray.get(ref)
    assert workflow.get_status("w5") == workflow.WorkflowStatus.CANCELED
    workflow.delete("w5")
    assert "w5" not in [w for w, _ in workflow.list_all()]
    with pytest.raises(workflow.WorkflowNotFoundError):
        workflow.get_status("w5")
