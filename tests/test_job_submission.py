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
