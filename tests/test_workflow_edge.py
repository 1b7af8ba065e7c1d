"""Workflow edge cases (reference test models: python/ray/workflow/tests/test_basic_workflows*.py
(nested DAG outputs, step results checkpointed so a resumed workflow does not re-run finished
steps), test_workflow_manager.py (list_all / get_status))."""
import pytest

import ray_community_amd as ray
from ray_community_amd import workflow


@pytest.fixture
def session(tmp_path):
    ray.init(num_cpus=2, storage=str(tmp_path / "wf"))
    yield tmp_path
    ray.shutdown()


def test_diamond_dag_and_status(session):
    @ray.remote
    def src(x):
        return x + 1

    @ray.remote
    def left(x):
        return x * 2

    @ray.remote
    def right(x):
        return x * 3

    @ray.remote
    def join(a, b):
        return a + b

    s = src.bind(1)
    dag = join.bind(left.bind(s), right.bind(s))
    assert workflow.run(dag, workflow_id="diamond") == 2 * 2 + 2 * 3
    assert workflow.get_status("diamond") == workflow.WorkflowStatus.SUCCESSFUL
    assert workflow.get_output("diamond") == 10
    assert "diamond" in {wid for wid, _ in workflow.list_all()}


def test_resume_does_not_rerun_finished_steps(session):
    marker = session / "count"
    fail_flag = session / "fail"
    fail_flag.write_text("1")

    @ray.remote
    def counted(path):
        n = int(open(path).read()) if __import__("os").path.exists(path) else 0
        open(path, "w").write(str(n + 1))
        return n + 1

    @ray.remote
    def maybe_fail(x, flag):
        if open(flag).read() == "1":
            raise RuntimeError("injected")
        return x * 10

    dag = maybe_fail.bind(counted.bind(str(marker)), str(fail_flag))
    with pytest.raises(Exception):
        workflow.run(dag, workflow_id="resumable")
    assert marker.read_text() == "1"
    fail_flag.write_text("0")
    assert workflow.resume("resumable") == 10
    assert marker.read_text() == "1"                        # the checkpointed step was not re-run
