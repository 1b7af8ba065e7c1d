"""Job submission (reference tests: dashboard/modules/job/tests/test_sdk.py, test_job_manager.py)."""
import asyncio
import sys

import pytest

import ray_community_amd as ray
from ray_community_amd.job_submission import JobStatus, JobSubmissionClient


def test_job_lifecycle(shutdown_only, tmp_path):
    ray.init(num_cpus=2)
    script = tmp_path / "job.py"
    script.write_text(
        "import os, ray_community_amd as ray\n"
        "ray.init()\n"
        "@ray.remote\n"
        "def sq(x):\n"
        "    return x * x\n"
        "print('result', sum(ray.get([sq.remote(i) for i in range(5)])), os.environ.get('MY_VAR'))\n")
    client = JobSubmissionClient()
    sid = client.submit_job(entrypoint=f"{sys.executable} job.py",
                            runtime_env={"working_dir": str(tmp_path), "env_vars": {"MY_VAR": "abc"}},
                            metadata={"owner": "test"})
    assert client.wait_until_finish(sid, 120) == JobStatus.SUCCEEDED, client.get_job_logs(sid)
    assert "result 30 abc" in client.get_job_logs(sid)
    info = client.get_job_info(sid)
    assert info.metadata == {"owner": "test"} and info.driver_exit_code == 0

    bad = client.submit_job(entrypoint=f"{sys.executable} -c 'import sys; sys.exit(3)'")
    assert client.wait_until_finish(bad, 60) == JobStatus.FAILED
    assert client.get_job_info(bad).driver_exit_code == 3

    slow = client.submit_job(entrypoint="sleep 30", submission_id="my-sleeper")
    assert slow == "my-sleeper"
    with pytest.raises(Exception):
        client.submit_job(entrypoint="true", submission_id="my-sleeper")
    assert client.stop_job(slow)
    assert client.wait_until_finish(slow, 30) == JobStatus.STOPPED
    assert {j.submission_id for j in client.list_jobs()} >= {sid, bad, slow}
    assert client.delete_job(slow)
    assert slow not in {j.submission_id for j in client.list_jobs()}

    tail = client.submit_job(entrypoint="echo one; echo two")

    async def collect():
        return "".join([c async for c in client.tail_job_logs(tail)])

    assert "two" in asyncio.run(collect())


def test_job_rest_api_over_http(shutdown_only, tmp_path):
    """JobSubmissionClient("http://127.0.0.1:<dashboard port>") drives the dashboard's job REST API
    (POST /api/jobs/, GET /api/jobs/{id}[/logs], POST /api/jobs/{id}/stop, DELETE /api/jobs/{id})."""
    import requests

    ctx = ray.init(num_cpus=2, include_dashboard=True, dashboard_port=0)
    url = ctx.dashboard_url
    client = JobSubmissionClient(url)
    sid = client.submit_job(entrypoint=f"{sys.executable} -c \"print('hello from http job')\"",
                            metadata={"via": "rest"})
    assert client.wait_until_finish(sid, 120) == JobStatus.SUCCEEDED
    assert "hello from http job" in client.get_job_logs(sid)
    assert client.get_job_info(sid).metadata == {"via": "rest"}
    slow = client.submit_job(entrypoint="sleep 30", submission_id="rest-sleeper")
    assert slow == "rest-sleeper" and client.get_job_status(slow) == JobStatus.RUNNING
    with pytest.raises(RuntimeError):
        client.delete_job(slow)  # not terminal yet
    assert client.stop_job(slow)
    assert client.wait_until_finish(slow, 30) == JobStatus.STOPPED
    assert {j.submission_id for j in client.list_jobs()} >= {sid, slow}
    assert client.delete_job(slow)
    assert requests.get(f"{url}/api/jobs/rest-sleeper", timeout=10).status_code == 404
    r = requests.post(f"{url}/api/jobs/", json={"entrypoint": "true", "submission_id": sid}, timeout=10)
    assert r.status_code == 400  # duplicate submission id


def test_entrypoint_resources_are_reserved_while_the_driver_runs(shutdown_only, tmp_path):
    import time

    ray.init(num_cpus=4, resources={"slot": 1})
    client = JobSubmissionClient()
    flag = tmp_path / "release"
    code = (f"import os, time\n"
            f"while not os.path.exists({str(flag)!r}): time.sleep(0.05)\n")
    (tmp_path / "hold.py").write_text(code)
    first = client.submit_job(entrypoint=f"{sys.executable} {tmp_path / 'hold.py'}", entrypoint_num_cpus=1,
                              entrypoint_resources={"slot": 1})
    deadline = time.time() + 60
    while client.get_job_status(first) != JobStatus.RUNNING and time.time() < deadline:
        time.sleep(0.1)
    assert client.get_job_status(first) == JobStatus.RUNNING
    assert ray.available_resources().get("slot", 0) == 0  # held by the running driver
    second = client.submit_job(entrypoint=f"{sys.executable} -c 'print(1)'", entrypoint_resources={"slot": 1})
    time.sleep(1.0)
    assert client.get_job_status(second) == JobStatus.PENDING  # waits for the slot
    flag.write_text("go")
    assert client.wait_until_finish(first, 60) == JobStatus.SUCCEEDED
    assert client.wait_until_finish(second, 60) == JobStatus.SUCCEEDED
    third = client.submit_job(entrypoint=f"{sys.executable} -c 'print(1)'", entrypoint_resources={"slot": 5})
    time.sleep(0.5)
    assert client.stop_job(third) and client.get_job_status(third) == JobStatus.STOPPED


def test_entrypoint_gpus_map_through_parent_mask(shutdown_only, tmp_path, monkeypatch):
    """A head started with HIP_VISIBLE_DEVICES=4,5 owns logical GPUs 0,1 = physical 4,5: a job
    reserving one GPU must see a PHYSICAL id (4 or 5), not the logical 0 (which would select
    physical GPU 0). ROCR_VISIBLE_DEVICES, which the HIP ids index into, is passed on unchanged."""
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,5")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    ray.init(num_cpus=2, num_gpus=2)
    client = JobSubmissionClient()
    sid = client.submit_job(
        entrypoint=f"{sys.executable} -c \"import os; print('VIS', os.environ.get('HIP_VISIBLE_DEVICES'), "
                   f"os.environ.get('ROCR_VISIBLE_DEVICES'))\"",
        entrypoint_num_gpus=1)
    assert client.wait_until_finish(sid, 120) == JobStatus.SUCCEEDED, client.get_job_logs(sid)
    line = [ln for ln in client.get_job_logs(sid).splitlines() if ln.startswith("VIS")][0]
    _, hip, rocr = line.split()
    assert hip in ("4", "5"), line
    assert rocr == "0,1,2,3,4,5,6,7"
