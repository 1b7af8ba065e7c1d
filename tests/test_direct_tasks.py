"""Normal tasks over leased workers (``_private/direct_transport.TaskLeaseChannel``; reference:
``src/ray/core_worker/transport/normal_task_submitter.cc`` + ``NodeManager::HandleRequestWorkerLease``):
results, worker-death retries and verdicts, application-error retries, cancellation, escaping
caller-owned results, nested submission, the state API, lease return, lineage of leased outputs."""
import os
import time

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import exceptions as exc


@pytest.fixture
def ray4():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _head():
    from ray_community_amd._private import worker

    return worker._state["head"]


def _wait_for(pred, timeout=10.0):
    t = time.time()
    while time.time() - t < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


@ray.remote
def inc(x):
    return x + 1


def test_burst_goes_over_leases_and_leases_are_returned(ray4):
    head = _head()
    n0 = len(head.tasks)
    refs = [inc.remote(i) for i in range(300)]
    assert ray.get(refs) == list(range(1, 301))
    # the head ran (almost) none of them itself: the burst went over leased workers
    assert len(head.tasks) - n0 < 30
    assert _wait_for(lambda: not head.leases)
    assert _wait_for(lambda: ray.available_resources().get("CPU") == 4.0)


def test_dependencies_between_owned_results(ray4):
    a = [inc.remote(i) for i in range(20)]
    b = [inc.remote(x) for x in a]
    assert ray.get(b) == [i + 2 for i in range(20)]


@ray.remote
def add(a, b):
    return a + b


def test_owned_result_escapes_to_head_scheduled_task(ray4):
    r = [inc.remote(i) for i in range(5)]
    # SPREAD tasks are scheduled by the head: the owned inputs are published to it
    out = [add.options(scheduling_strategy="SPREAD").remote(r[i], r[i + 1]) for i in range(4)]
    assert ray.get(out) == [3, 5, 7, 9]
    box = ray.put([r[0]])  # a ref nested in a put object escapes too
    assert ray.get(ray.get(box)[0]) == 1


@ray.remote
def nested(n):
    return sum(ray.get([inc.remote(i) for i in range(n)]))


def test_nested_submission_from_leased_workers(ray4):
    assert ray.get([nested.remote(8) for _ in range(6)]) == [36] * 6


@ray.remote(max_retries=2)
def die_once(path):
    if not os.path.exists(path):
        open(path, "w").close()
        os._exit(1)
    return "survived"


def test_worker_death_retries(ray4, tmp_path):
    marks = [str(tmp_path / f"m{i}") for i in range(3)]
    assert ray.get([die_once.remote(m) for m in marks]) == ["survived"] * 3


@ray.remote(max_retries=0)
def die_always():
    os._exit(1)


def test_worker_death_without_retries_fails(ray4):
    refs = [die_always.remote() for _ in range(2)]
    for r in refs:
        with pytest.raises(exc.WorkerCrashedError):
            ray.get(r, timeout=30)


@ray.remote(max_retries=3, retry_exceptions=True)
def flaky(path):
    n = int(open(path).read() or 0) if os.path.exists(path) else 0
    with open(path, "w") as f:
        f.write(str(n + 1))
    if n < 2:
        raise ValueError("not yet")
    return n


def test_application_errors_retry(ray4, tmp_path):
    paths = [str(tmp_path / f"c{i}") for i in range(3)]
    assert ray.get([flaky.remote(p) for p in paths]) == [2, 2, 2]


@ray.remote
def boom():
    raise KeyError("nope")


def test_application_error_propagates(ray4):
    refs = [boom.remote() for _ in range(3)]
    with pytest.raises(KeyError):
        ray.get(refs[0])
    with pytest.raises(exc.RayTaskError):
        ray.get(refs[1])


@ray.remote
def sleepy(t):
    time.sleep(t)
    return t


def test_cancel_queued_and_running(ray4):
    running = [sleepy.remote(30) for _ in range(4)]
    queued = sleepy.remote(0)
    time.sleep(0.5)
    ray.cancel(queued)
    with pytest.raises(exc.TaskCancelledError):
        ray.get(queued, timeout=10)
    for r in running:
        ray.cancel(r, force=True)
    for r in running:
        with pytest.raises(exc.TaskCancelledError):
            ray.get(r, timeout=30)


def test_state_api_sees_leased_tasks(ray4):
    from ray_community_amd.util import state

    ray.get([inc.options(name="leased_inc").remote(i) for i in range(10)])
    assert _wait_for(lambda: sum(1 for t in state.list_tasks()
                                 if t["name"] == "leased_inc" and t["state"] == "FINISHED") >= 9)
    kinds = {t["type"] for t in state.list_tasks() if t["name"] == "leased_inc"}
    assert kinds <= {"NORMAL_TASK"}


def test_blocked_leased_worker_lends_its_cpu():
    ray.init(num_cpus=2)
    try:
        @ray.remote
        def outer(n):
            return sum(ray.get([inc.remote(i) for i in range(n)]))

        # 2 CPUs, 2 outer tasks that wait on inner tasks: only works if waiting lends the CPU back
        assert ray.get([outer.remote(4), outer.remote(4)], timeout=60) == [10, 10]
    finally:
        ray.shutdown()


@ray.remote(max_retries=2, resources={"slot": 1})
def big_slot(path, seed):
    with open(path, "a") as f:
        f.write("x")
    return np.full(200_000, seed, dtype=np.int64)  # shm-resident: registered with the head


def test_leased_output_is_reconstructed_when_its_node_dies(ray_start_cluster, tmp_path):
    cluster = ray_start_cluster
    cluster.add_node(num_cpus=2)
    n2 = cluster.add_node(num_cpus=2, resources={"slot": 2})
    runs = tmp_path / "runs"
    runs.write_text("")
    refs = [big_slot.remote(str(runs), s) for s in (5, 6)]
    assert [int(ray.get(r)[0]) for r in refs] == [5, 6]
    assert open(runs).read() == "xx"
    cluster.add_node(num_cpus=2, resources={"slot": 2})
    cluster.remove_node(n2)
    out = ray.get(refs[1], timeout=60)  # recomputed on the new node from its lineage
    assert int(out[-1]) == 6
    assert open(runs).read().count("x") >= 3


def test_pipelined_actor_calls_do_not_deadlock_on_full_sockets(shutdown_only):
    """Tens of thousands of direct actor calls submitted without waiting fill the caller->actor
    socket. The caller must keep reading replies while a send is blocked: the native frame writer
    once blocked with the GIL held (and the channel sent under its lock), freezing the reader
    thread, so caller and actor both stopped reading (core microbenchmark 1:1 actor calls async)."""
    import threading

    ray.init(num_cpus=2, include_dashboard=False)

    @ray.remote
    class Echo:
        def v(self, x=b"ok"):
            return x

    a = Echo.remote()
    ray.get(a.v.remote())
    done = []

    def work():
        for _ in range(6):
            refs = [a.v.remote(b"x" * 200) for _ in range(4000)]
            assert ray.get(refs, timeout=120)[-1] == b"x" * 200
        done.append(True)

    t = threading.Thread(target=work, daemon=True)
    t.start()
    t.join(150)
    assert done, "pipelined actor calls stalled"


def test_async_actor_calls_start_in_submission_order(shutdown_only):
    """Async actors read their direct connections on the actor's event loop: calls from one caller
    still start in submission order, and cancellation of a queued call works."""
    import asyncio

    ray.init(num_cpus=2, include_dashboard=False)

    @ray.remote
    class Rec:
        def __init__(self):
            self.seen = []

        async def add(self, i):
            self.seen.append(i)
            await asyncio.sleep(0)
            return i

        async def slow(self):
            await asyncio.sleep(30)

        async def get(self):
            return self.seen

    r = Rec.remote()
    refs = [r.add.remote(i) for i in range(2000)]
    assert ray.get(refs)[-1] == 1999
    assert ray.get(r.get.remote()) == list(range(2000))
    s = r.slow.remote()
    time.sleep(0.3)
    ray.cancel(s)
    with pytest.raises((exc.TaskCancelledError, exc.RayTaskError)):
        ray.get(s, timeout=20)


def test_leased_worker_of_a_dead_driver_is_killed(tmp_path):
    """A second driver leases a worker, starts a long task on it and dies. The head cannot know
    whether the worker is still running that orphan task, so it kills the worker instead of
    returning it (busy) to the idle pool; the cluster keeps serving the remaining driver."""
    import subprocess
    import sys

    import psutil

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    env.pop("RAY_ADDRESS", None)
    env["RCA_TEMP_DIR"] = str(tmp_path)
    head = subprocess.Popen([sys.executable, "-m", "ray_community_amd", "start", "--head", "--block", "--num-cpus",
                             "1", "--temp-dir", str(tmp_path)], cwd=root, env=env, stdout=subprocess.DEVNULL,
                            stderr=subprocess.STDOUT)
    pidfile = tmp_path / "orphan.pid"
    try:
        drv = ("import os, sys, time; sys.path.insert(0, %r)\n"
               "import ray_community_amd as ray\n"
               "for _ in range(600):\n"
               "    try:\n"
               "        ray.init(address='auto'); break\n"
               "    except Exception:\n"
               "        time.sleep(0.2)\n"
               "@ray.remote\n"
               "def orphan(path):\n"
               "    open(path + '.tmp', 'w').write(str(os.getpid())); os.replace(path + '.tmp', path)\n"
               "    time.sleep(300)\n"
               "orphan.remote(%r)\n"
               "while not os.path.exists(%r): time.sleep(0.05)\n"
               "os._exit(0)\n") % (root, str(pidfile), str(pidfile))
        r = subprocess.run([sys.executable, "-c", drv], cwd=root, env=env, capture_output=True, text=True,
                           timeout=180)
        assert r.returncode == 0, r.stderr
        pid = int(pidfile.read_text())
        def alive(p):  # the pid can vanish between any two psutil calls
            try:
                return psutil.Process(p).status() != psutil.STATUS_ZOMBIE
            except psutil.NoSuchProcess:
                return False

        deadline = time.time() + 20
        while time.time() < deadline and alive(pid):
            time.sleep(0.1)
        assert not alive(pid), "orphan worker still running"
        drv2 = ("import sys; sys.path.insert(0, %r)\n"
                "import ray_community_amd as ray\n"
                "ray.init(address='auto')\n"
                "@ray.remote\n"
                "def one():\n"
                "    return 1\n"
                "assert ray.get(one.remote(), timeout=60) == 1\n"
                "ray.shutdown()\n") % root
        r = subprocess.run([sys.executable, "-c", drv2], cwd=root, env=env, capture_output=True, text=True,
                           timeout=180)
        assert r.returncode == 0, r.stderr
    finally:
        head.terminate()
        try:
            head.wait(timeout=30)
        except subprocess.TimeoutExpired:
            head.kill()
