"""Job submission (reference: ``python/ray/job_submission``, ``dashboard/modules/job/``).

``JobSubmissionClient`` talks to a detached ``JobManager`` actor of the running session. Each job
is its entrypoint shell command started as a child process group of that actor, with
``RCA_ADDRESS`` pointing at the session so the job's ``init()`` joins the same cluster, the job's
runtime_env applied (env_vars, working_dir as cwd, py_modules on PYTHONPATH), and stdout/stderr
captured to a per-job log file under the session's ``logs/`` directory.
"""
from __future__ import annotations

import asyncio
import dataclasses
import enum
import json
import os
import signal
import subprocess
import threading
import time
import uuid
from typing import Any, AsyncIterator, Dict, List, Optional

_MANAGER = "_rca_job_manager"
_NS = "_rca_jobs"


class JobStatus(str, enum.Enum):
    PENDING = "PENDING"
    RUNNING = "RUNNING"
    STOPPED = "STOPPED"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"

    def is_terminal(self) -> bool:
        return self in (JobStatus.STOPPED, JobStatus.SUCCEEDED, JobStatus.FAILED)

    def __str__(self):
        return self.value


class JobType(str, enum.Enum):
    SUBMISSION = "SUBMISSION"
    DRIVER = "DRIVER"


@dataclasses.dataclass
class JobInfo:
    status: JobStatus
    entrypoint: str
    message: Optional[str] = None
    error_type: Optional[str] = None
    start_time: Optional[int] = None
    end_time: Optional[int] = None
    metadata: Optional[Dict[str, str]] = None
    runtime_env: Optional[Dict[str, Any]] = None
    driver_exit_code: Optional[int] = None
    submission_id: Optional[str] = None
    job_id: Optional[str] = None
    type: JobType = JobType.SUBMISSION
    entrypoint_num_cpus: Optional[float] = None
    entrypoint_num_gpus: Optional[float] = None
    entrypoint_resources: Optional[Dict[str, float]] = None


JobDetails = JobInfo


@dataclasses.dataclass
class DriverInfo:
    """The driver process of a job (reference ``dashboard/modules/job/pydantic_models.py``
    ``DriverInfo``): its job id, the node address it runs on and its pid."""
    id: str
    node_ip_address: str
    pid: str


class _EntrypointReservation:
    """Holds a job's ``entrypoint_num_cpus / _num_gpus / _memory / _resources`` for as long as its
    driver runs (reference: the job supervisor actor is scheduled with them); the GPUs it was
    given become the driver's visible devices."""

    def gpu_ids(self):
        from ._private.worker import get_gpu_ids

        return [str(g) for g in get_gpu_ids()]

    def device_env(self):
        """The device-visibility variables the driver must run with to see exactly this holder's
        GPUs: the holder's own ``HIP_VISIBLE_DEVICES`` -- already mapped through the head's parent
        mask by the worker pool (``_private/head.py::worker_hip_visible_devices``), i.e. PHYSICAL
        ids when the head was started with ``HIP_VISIBLE_DEVICES=4,5`` -- and the
        ``ROCR_VISIBLE_DEVICES`` it indexes into. Empty when no GPU was reserved."""
        if not self.gpu_ids():
            return {}
        out = {}
        hip = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
        if hip:
            out["HIP_VISIBLE_DEVICES"] = out["CUDA_VISIBLE_DEVICES"] = hip
        rocr = os.environ.get("ROCR_VISIBLE_DEVICES")
        if rocr is not None:
            out["ROCR_VISIBLE_DEVICES"] = rocr
        return out


class JobManager:
    """Detached actor owning the job processes."""

    def __init__(self, address: str, logs_dir: str):
        self.address = address
        self.logs_dir = logs_dir
        os.makedirs(logs_dir, exist_ok=True)
        self.jobs: Dict[str, Dict] = {}
        self.procs: Dict[str, subprocess.Popen] = {}
        self.holders: Dict[str, Any] = {}  # sid -> the actor reserving the entrypoint's resources
        self.lock = threading.Lock()
        threading.Thread(target=self._monitor, daemon=True).start()

    def _monitor(self):
        while True:
            time.sleep(0.05)
            with self.lock:
                for sid, p in list(self.procs.items()):
                    rc = p.poll()
                    if rc is None:
                        continue
                    j = self.jobs[sid]
                    j["driver_exit_code"] = rc
                    j["end_time"] = int(time.time() * 1000)
                    if j["status"] == JobStatus.STOPPED:
                        j["message"] = "Job was intentionally stopped."
                    elif rc == 0:
                        j["status"] = JobStatus.SUCCEEDED
                        j["message"] = "Job finished successfully."
                    else:
                        j["status"] = JobStatus.FAILED
                        j["error_type"] = "JOB_ENTRYPOINT_COMMAND_ERROR"
                        j["message"] = f"Job entrypoint command failed with exit code {rc}"
                    del self.procs[sid]
                    self._release(sid)

    def _release(self, sid: str) -> None:
        holder = self.holders.pop(sid, None)
        if holder is not None:
            from ._private.worker import kill

            try:
                kill(holder)
            except Exception:  # noqa: BLE001 -- already gone
                pass

    def _reserve(self, resources: Dict):
        """An actor holding the requested entrypoint resources, and its GPU ids (blocks until the
        cluster can place it: the job stays PENDING meanwhile)."""
        from . import remote
        from ._private.worker import get

        ncpu = resources.get("entrypoint_num_cpus") or 0
        ngpu = resources.get("entrypoint_num_gpus") or 0
        custom = dict(resources.get("entrypoint_resources") or {})
        mem = resources.get("entrypoint_memory")
        opts = {"num_cpus": ncpu, "num_gpus": ngpu, "resources": custom}
        if mem:
            opts["memory"] = mem
        holder = remote(_EntrypointReservation).options(**opts).remote()
        return holder, get(holder.device_env.remote())

    def submit(self, entrypoint: str, submission_id: Optional[str], runtime_env: Optional[Dict],
               metadata: Optional[Dict], resources: Dict) -> str:
        sid = submission_id or f"raysubmit_{uuid.uuid4().hex[:16]}"
        with self.lock:
            if sid in self.jobs:
                raise ValueError(f"Job with submission_id {sid} already exists. Please use a different submission_id.")
            renv = dict(runtime_env or {})
            env = dict(os.environ)
            env["RCA_ADDRESS"] = self.address
            env["RAY_ADDRESS"] = self.address
            env["RCA_JOB_SUBMISSION_ID"] = sid
            env.pop("RCA_WORKER_ID", None)
            for k, v in (renv.get("env_vars") or {}).items():
                env[str(k)] = str(v)
            cwd = os.getcwd()
            if renv.get("working_dir"):
                from .runtime_env import prepare_working_dir

                cwd = prepare_working_dir(str(renv["working_dir"]), os.path.dirname(self.logs_dir))
            paths = [p if os.path.isdir(p) else os.path.dirname(p) for p in renv.get("py_modules") or []]
            pkg_parent = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            env["PYTHONPATH"] = os.pathsep.join(paths + [cwd, pkg_parent] + ([env["PYTHONPATH"]]
                                                                             if env.get("PYTHONPATH") else []))
            log = os.path.join(self.logs_dir, f"job-driver-{sid}.log")
            self.jobs[sid] = {"status": JobStatus.PENDING, "entrypoint": entrypoint, "submission_id": sid,
                              "metadata": dict(metadata or {}), "runtime_env": renv,
                              "start_time": int(time.time() * 1000), "log": log, **resources}
            if not any(resources.get(k) for k in ("entrypoint_num_cpus", "entrypoint_num_gpus",
                                                  "entrypoint_resources", "entrypoint_memory")):
                self._launch(sid, entrypoint, cwd, env, log)
                return sid
        # reserved entrypoint resources: PENDING until they are placed, then the driver starts
        threading.Thread(target=self._launch_reserved, args=(sid, entrypoint, cwd, env, log, resources),
                         daemon=True).start()
        return sid

    def _launch(self, sid, entrypoint, cwd, env, log) -> None:
        with open(log, "ab") as f:
            p = subprocess.Popen(entrypoint, shell=True, cwd=cwd, env=env, stdout=f, stderr=subprocess.STDOUT,
                                 stdin=subprocess.DEVNULL, start_new_session=True)
        self.procs[sid] = p
        self.jobs[sid]["status"] = JobStatus.RUNNING
        self.jobs[sid]["job_id"] = f"{p.pid:08x}"

    def _launch_reserved(self, sid, entrypoint, cwd, env, log, resources) -> None:
        try:
            holder, dev_env = self._reserve(resources)
        except Exception as e:  # noqa: BLE001 -- an unplaceable request fails the job
            with self.lock:
                j = self.jobs[sid]
                j["status"], j["error_type"] = JobStatus.FAILED, "JOB_SUPERVISOR_ACTOR_START_FAILURE"
                j["message"] = f"could not reserve the entrypoint resources: {e}"
                j["end_time"] = int(time.time() * 1000)
            return
        if dev_env:  # the driver sees exactly the GPUs reserved for it (physical ids, not logical)
            env = dict(env, **dev_env)
        with self.lock:
            self.holders[sid] = holder
            if self.jobs[sid]["status"] == JobStatus.STOPPED:  # stopped while pending
                self._release(sid)
                return
            self._launch(sid, entrypoint, cwd, env, log)

    def info(self, sid: str) -> Optional[Dict]:
        with self.lock:
            j = self.jobs.get(sid)
            return None if j is None else {k: v for k, v in j.items() if k != "log"}

    def list(self) -> List[Dict]:
        with self.lock:
            return [{k: v for k, v in j.items() if k != "log"} for j in self.jobs.values()]

    def logs(self, sid: str, offset: int = 0) -> Optional[str]:
        j = self.jobs.get(sid)
        if j is None:
            return None
        try:
            with open(j["log"], "rb") as f:
                f.seek(offset)
                return f.read().decode(errors="replace")
        except FileNotFoundError:
            return ""

    def stop(self, sid: str) -> bool:
        with self.lock:
            p = self.procs.get(sid)
            if p is None:
                j = self.jobs.get(sid)
                if j is not None and j["status"] == JobStatus.PENDING:  # still waiting for its resources
                    j["status"], j["end_time"] = JobStatus.STOPPED, int(time.time() * 1000)
                    j["message"] = "Job was intentionally stopped."
                    return True
                return False
            self.jobs[sid]["status"] = JobStatus.STOPPED
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            return True
        deadline = time.time() + 3
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        return True

    def delete(self, sid: str) -> bool:
        with self.lock:
            j = self.jobs.get(sid)
            if j is None:
                raise ValueError(f"job {sid} does not exist")
            if not j["status"].is_terminal():
                raise RuntimeError(f"Attempted to delete job '{sid}', but it is in a non-terminal state "
                                   f"{j['status']}.")
            del self.jobs[sid]
            return True


def _to_info(d: Dict) -> JobInfo:
    fields = {f.name for f in dataclasses.fields(JobInfo)}
    return JobInfo(**{k: v for k, v in d.items() if k in fields})


def _job_manager(create: bool = True):
    """The session's detached JobManager actor (created on first use)."""
    from ._private import worker as w
    from .actor import ActorClass

    try:
        return w.get_actor(_MANAGER, namespace=_NS)
    except ValueError:
        if not create:
            raise
        core = w._core()
        logs = os.path.join(core.session_dir or "/tmp/rca", "logs")
        addr = w._state.get("address")
        return ActorClass(JobManager, {"name": _MANAGER, "namespace": _NS, "lifetime": "detached",
                                       "num_cpus": 0, "max_concurrency": 64,
                                       "get_if_exists": True}).remote(addr, logs)


def _jsonable_job(d: Dict) -> Dict:
    out = dict(d)
    for k, v in out.items():
        if isinstance(v, enum.Enum):
            out[k] = v.value
    return out


class JobSubmissionClient:
    """Submit and manage jobs.

    ``address="http://host:8265"`` talks to the dashboard's job REST API (reference
    ``dashboard/modules/job/job_head.py``: ``POST /api/jobs/``, ``GET /api/jobs/{id}``,
    ``POST /api/jobs/{id}/stop``, ``DELETE /api/jobs/{id}``, ``GET /api/jobs/{id}/logs``); any other
    address (a session socket, ``"auto"``, ``None``) joins the session and drives the JobManager
    actor directly.
    """

    def __init__(self, address: Optional[str] = None, create_cluster_if_needed: bool = False, cookies=None,
                 metadata=None, headers=None, verify=None):
        self._http = None
        if address and address.startswith(("http://", "https://")):
            import requests

            self._http = address.rstrip("/")
            self._session = requests.Session()
            if headers:
                self._session.headers.update(headers)
            if cookies:
                self._session.cookies.update(cookies)
            r = self._session.get(self._http + "/api/version", timeout=10)
            r.raise_for_status()
            return
        from ._private import worker as w

        if not w.is_initialized():
            if address in (None, "auto") and not create_cluster_if_needed:
                w.init(address=address if address != "auto" else None, ignore_reinit_error=True)
            else:
                w.init(address=None if address in (None, "auto", "local") else address, ignore_reinit_error=True)
        self._mgr = _job_manager()
        self._get = w.get

    # ------------------------------------------------------------------ HTTP transport
    def _req(self, method: str, path: str, **kw):
        r = self._session.request(method, self._http + path, timeout=60, **kw)
        if r.status_code == 404:
            raise RuntimeError(r.json().get("error", f"{path} not found") if r.headers.get(
                "content-type", "").startswith("application/json") else f"{path} not found")
        if r.status_code >= 400:
            raise RuntimeError(f"{method} {path} failed ({r.status_code}): {r.text}")
        return r.json()

    def submit_job(self, *, entrypoint: str, job_id: Optional[str] = None, runtime_env: Optional[Dict] = None,
                   metadata: Optional[Dict[str, str]] = None, submission_id: Optional[str] = None,
                   entrypoint_num_cpus: Optional[float] = None, entrypoint_num_gpus: Optional[float] = None,
                   entrypoint_resources: Optional[Dict[str, float]] = None, entrypoint_memory: Optional[int] = None,
                   **kw) -> str:
        from .runtime_env import validate

        res = {"entrypoint_num_cpus": entrypoint_num_cpus, "entrypoint_num_gpus": entrypoint_num_gpus,
               "entrypoint_resources": entrypoint_resources, "entrypoint_memory": entrypoint_memory}
        if self._http:
            body = {"entrypoint": entrypoint, "submission_id": submission_id or job_id,
                    "runtime_env": runtime_env, "metadata": metadata, **res}
            return self._req("POST", "/api/jobs/", json=body)["submission_id"]
        return self._get(self._mgr.submit.remote(entrypoint, submission_id or job_id, validate(runtime_env),
                                                 metadata, res))

    def get_job_info(self, job_id: str) -> JobInfo:
        if self._http:
            d = self._req("GET", f"/api/jobs/{job_id}")
            d["status"] = JobStatus(d["status"])
            return _to_info(d)
        d = self._get(self._mgr.info.remote(job_id))
        if d is None:
            raise RuntimeError(f"Job {job_id} does not exist.")
        return _to_info(d)

    def get_job_status(self, job_id: str) -> JobStatus:
        return self.get_job_info(job_id).status

    def list_jobs(self) -> List[JobDetails]:
        if self._http:
            out = []
            for d in self._req("GET", "/api/jobs/"):
                d["status"] = JobStatus(d["status"])
                out.append(_to_info(d))
            return out
        return [_to_info(d) for d in self._get(self._mgr.list.remote())]

    def get_job_logs(self, job_id: str) -> str:
        if self._http:
            return self._req("GET", f"/api/jobs/{job_id}/logs")["logs"]
        out = self._get(self._mgr.logs.remote(job_id, 0))
        if out is None:
            raise RuntimeError(f"Job {job_id} does not exist.")
        return out

    async def tail_job_logs(self, job_id: str) -> AsyncIterator[str]:
        offset = 0
        while True:
            if self._http:
                loop = asyncio.get_running_loop()
                d = await loop.run_in_executor(None, lambda: self._req("GET", f"/api/jobs/{job_id}/logs",
                                                                       params={"offset": offset}))
                chunk = d["logs"]
                info = await loop.run_in_executor(None, lambda: self._req("GET", f"/api/jobs/{job_id}"))
            else:
                chunk = await self._mgr.logs.remote(job_id, offset)
                info = await self._mgr.info.remote(job_id)
            if chunk:
                offset += len(chunk.encode())
                yield chunk
            if info is None or JobStatus(info["status"]).is_terminal():
                rest = (self._req("GET", f"/api/jobs/{job_id}/logs", params={"offset": offset})["logs"]
                        if self._http else await self._mgr.logs.remote(job_id, offset))
                if rest:
                    yield rest
                return
            await asyncio.sleep(0.1)

    def stop_job(self, job_id: str) -> bool:
        if self._http:
            return self._req("POST", f"/api/jobs/{job_id}/stop")["stopped"]
        return self._get(self._mgr.stop.remote(job_id))

    def delete_job(self, job_id: str) -> bool:
        if self._http:
            return self._req("DELETE", f"/api/jobs/{job_id}")["deleted"]
        return self._get(self._mgr.delete.remote(job_id))

    def wait_until_finish(self, job_id: str, timeout_s: float = 600) -> JobStatus:
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            st = self.get_job_status(job_id)
            if st.is_terminal():
                return st
            time.sleep(0.1)
        raise TimeoutError(f"job {job_id} did not finish in {timeout_s}s")


__all__ = ["JobSubmissionClient", "JobStatus", "JobInfo", "JobDetails", "JobType", "DriverInfo"]
