"""Actor tests (modelled on reference python/ray/tests/test_actor*.py)."""
import asyncio
import os
import threading
import time

import pytest

import ray_community_amd as ray
from ray_community_amd import exceptions as exc


@ray.remote
class Counter:
    def __init__(self, start=0):
        self.n = start

    def inc(self, k=1):
        self.n += k
        return self.n

    def get(self):
        return self.n

    def pid(self):
        return os.getpid()

    def fail(self):
        raise KeyError("nope")

    def die(self):
        os._exit(1)


def _alive(pid):
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("State:"):
                    return "Z" not in line.split()[1]
    except OSError:
        return False
    return True


def test_actor_basic_and_ordering(ray_start_regular):
    c = Counter.remote(10)
    refs = [c.inc.remote() for _ in range(50)]
    assert ray.get(refs) == list(range(11, 61))
    assert ray.get(c.get.remote()) == 60


def test_actor_error_keeps_actor_alive(ray_start_regular):
    c = Counter.remote()
    with pytest.raises(KeyError):
        ray.get(c.fail.remote())
    assert ray.get(c.inc.remote()) == 1


def test_actor_handle_passing(ray_start_regular):
    c = Counter.remote()

    @ray.remote
    def use(h):
        return ray.get(h.inc.remote(5))

    assert ray.get(use.remote(c)) == 5
    assert ray.get(c.get.remote()) == 5


def test_named_actor(ray_start_regular):
    c = Counter.options(name="ctr").remote()
    ray.get(c.inc.remote())
    h = ray.get_actor("ctr")
    assert ray.get(h.get.remote()) == 1
    with pytest.raises(ValueError):
        Counter.options(name="ctr").remote()
    h2 = Counter.options(name="ctr", get_if_exists=True).remote()
    assert ray.get(h2.get.remote()) == 1
    with pytest.raises(ValueError):
        ray.get_actor("nope")


def test_kill_actor(ray_start_regular):
    c = Counter.remote()
    ray.get(c.inc.remote())
    ray.kill(c)
    with pytest.raises(exc.RayActorError):
        ray.get(c.inc.remote(), timeout=10)


def test_actor_restart(ray_start_regular):
    c = Counter.options(max_restarts=1).remote()
    p1 = ray.get(c.pid.remote())
    with pytest.raises(exc.RayActorError):
        ray.get(c.die.remote())
    p2 = ray.get(c.pid.remote(), timeout=20)
    assert p1 != p2
    assert ray.get(c.get.remote()) == 0  # state re-initialised
    with pytest.raises(exc.RayActorError):
        ray.get(c.die.remote())
    with pytest.raises(exc.RayActorError):
        ray.get(c.get.remote(), timeout=10)


def test_actor_init_failure(ray_start_regular):
    @ray.remote
    class Bad:
        def __init__(self):
            raise RuntimeError("ctor")

        def f(self):
            return 1

    b = Bad.remote()
    with pytest.raises(exc.RayActorError):
        ray.get(b.f.remote(), timeout=10)


def test_async_actor(ray_start_regular):
    @ray.remote
    class A:
        def __init__(self):
            self.ev = None

        async def wait_and_get(self, t):
            await asyncio.sleep(t)
            return t

    a = A.remote()
    t0 = time.time()
    out = ray.get([a.wait_and_get.remote(0.5) for _ in range(20)])
    assert out == [0.5] * 20
    assert time.time() - t0 < 5  # concurrent, not 10 s


def test_threaded_actor(ray_start_regular):
    @ray.remote(max_concurrency=4)
    class T:
        def work(self):
            time.sleep(0.3)
            return threading.get_ident()

    t = T.remote()
    t0 = time.time()
    ids = ray.get([t.work.remote() for _ in range(4)])
    assert time.time() - t0 < 1.1
    assert len(set(ids)) > 1


def test_actor_method_num_returns(ray_start_regular):
    @ray.remote
    class M:
        @ray.method(num_returns=2)
        def two(self):
            return 1, 2

    m = M.remote()
    a, b = m.two.remote()
    assert ray.get([a, b]) == [1, 2]


def test_exit_actor(ray_start_regular):
    @ray.remote
    class E:
        def bye(self):
            ray.exit_actor()

        def ping(self):
            return 1

    e = E.remote()
    assert ray.get(e.ping.remote()) == 1
    ray.get(e.bye.remote())
    with pytest.raises(exc.RayActorError):
        ray.get(e.ping.remote(), timeout=10)


def test_actor_out_of_scope_is_killed(ray_start_regular):
    c = Counter.remote()
    pid = ray.get(c.pid.remote())
    del c
    deadline = time.time() + 10
    while time.time() < deadline:
        if not _alive(pid):
            break
        time.sleep(0.1)
    else:
        pytest.fail("actor process still alive after its handle went out of scope")


def test_detached_actor_survives_handle(ray_start_regular):
    c = Counter.options(name="det", lifetime="detached").remote()
    ray.get(c.inc.remote())
    del c
    time.sleep(0.5)
    assert ray.get(ray.get_actor("det").get.remote()) == 1


def test_actor_generator(ray_start_regular):
    @ray.remote
    class G:
        def stream(self, n):
            for i in range(n):
                yield i

    g = G.remote()
    assert [ray.get(r) for r in g.stream.remote(4)] == [0, 1, 2, 3]


def test_actor_gpu_assignment_without_gpus(ray_start_regular):
    @ray.remote
    class X:
        def gpus(self):
            return ray.get_gpu_ids()

    assert ray.get(X.remote().gpus.remote()) == []


def test_ready(ray_start_regular):
    c = Counter.remote()
    assert ray.get(c.__ray_ready__.remote()) is True


# ----------------------------------------------------------------------------- direct transport
def test_per_caller_ordering_with_unresolved_dependency(ray_start_regular):
    """An earlier call with an unresolved ObjectRef argument holds back only the same caller's
    later calls (submission order kept); another caller's calls are not blocked behind it."""

    @ray.remote
    class Log:
        def __init__(self):
            self.seen = []

        def add(self, tag, *_dep):
            self.seen.append(tag)
            return tag

        def seen_list(self):
            return list(self.seen)

    @ray.remote
    def slow(x):
        time.sleep(1.5)
        return x

    @ray.remote
    def other_caller(log):
        return ray.get(log.add.remote("B1"))

    log = Log.remote()
    ray.get(log.seen_list.remote())
    dep = slow.remote(0)
    a1 = log.add.remote("A1", dep)   # blocked on dep
    a2 = log.add.remote("A2")        # same caller: must run after A1
    t0 = time.time()
    assert ray.get(other_caller.remote(log)) == "B1"  # different caller: not blocked by A1
    assert time.time() - t0 < 1.3
    assert ray.get([a1, a2]) == ["A1", "A2"]
    seen = ray.get(log.seen_list.remote())
    assert seen.index("B1") < seen.index("A1") < seen.index("A2")


def test_direct_results_escape_to_tasks_and_puts(ray_start_regular):
    """Caller-owned results of direct actor calls passed on (as task args, nested in a put, in
    wait() mixed with head-managed refs) are published to the head transparently."""
    c = Counter.remote(100)

    @ray.remote
    def plus(x, y):
        return x + y

    @ray.remote
    def unwrap(lst):
        return ray.get(lst[0])

    r = c.inc.remote()           # pending while we pass it on
    assert ray.get(plus.remote(r, 1)) == 102
    nested = ray.put([c.inc.remote()])
    assert ray.get(unwrap.remote(nested)) == 102
    r2 = c.inc.remote()
    p = plus.remote(1, 2)
    ready, _ = ray.wait([r2, p], num_returns=2, timeout=30)
    assert len(ready) == 2 and ray.get(r2) == 103


def test_direct_call_retried_after_actor_restart(ray_start_regular):
    """The stream to a restarting actor breaks: in-flight calls with max_task_retries are re-sent
    to the new incarnation, calls without retries fail with ActorDiedError."""

    @ray.remote(max_restarts=1, max_task_retries=1)
    class Flaky:
        def __init__(self):
            self.calls = 0

        def pid(self):
            return os.getpid()

        def die_once(self, marker):
            if not os.path.exists(marker):
                open(marker, "w").close()
                os._exit(1)
            return "survived"

    import tempfile

    marker = os.path.join(tempfile.mkdtemp(), "m")
    f = Flaky.remote()
    pid0 = ray.get(f.pid.remote())
    assert ray.get(f.die_once.remote(marker), timeout=60) == "survived"
    assert ray.get(f.pid.remote()) != pid0
    g = Flaky.options(max_task_retries=0).remote()
    marker2 = os.path.join(tempfile.mkdtemp(), "m")
    with pytest.raises(exc.RayActorError):
        ray.get(g.die_once.remote(marker2), timeout=60)


def test_direct_calls_visible_in_state_api_and_timeline(ray_start_regular):
    from ray_community_amd.util import state

    c = Counter.remote()
    ray.get([c.inc.remote() for _ in range(5)])
    deadline = time.time() + 10
    names = []
    while time.time() < deadline:
        names = [t["name"] for t in state.list_tasks() if t["type"] == "ACTOR_TASK"]
        if names.count("Counter.inc") >= 5:
            break
        time.sleep(0.2)
    assert names.count("Counter.inc") >= 5
    assert any(e["name"] == "Counter.inc" for e in ray.timeline())


def test_concurrency_groups_threaded_and_async(ray_start_regular):
    """Methods in a concurrency group run on that group's own concurrency budget (reference
    test_concurrency_group.py): two 'io' calls overlap (group of 2) while 'compute' calls
    serialise (group of 1); async actors bound each group's coroutines the same way."""
    import time as _t

    @ray.remote(concurrency_groups={"io": 2, "compute": 1})
    class T:
        @ray.method(concurrency_group="io")
        def io(self):
            _t.sleep(0.6)
            return _t.time()

        @ray.method(concurrency_group="compute")
        def compute(self):
            _t.sleep(0.4)
            return _t.time()

    a = T.remote()
    ray.get(a.__ray_ready__.remote()) if hasattr(a, "__ray_ready__") else None
    t0 = _t.time()
    ray.get([a.io.remote(), a.io.remote()])
    assert _t.time() - t0 < 1.1  # overlapped
    t0 = _t.time()
    ray.get([a.compute.remote(), a.compute.remote()])
    assert _t.time() - t0 >= 0.75  # serialised

    import asyncio

    @ray.remote(concurrency_groups={"one": 1})
    class A:
        @ray.method(concurrency_group="one")
        async def solo(self):
            await asyncio.sleep(0.3)
            return 1

        async def free(self):
            await asyncio.sleep(0.3)
            return 2

    b = A.remote()
    ray.get(b.free.remote())
    t0 = _t.time()
    ray.get([b.solo.remote() for _ in range(3)])
    assert _t.time() - t0 >= 0.85  # one at a time
    t0 = _t.time()
    ray.get([b.free.remote() for _ in range(3)])
    assert _t.time() - t0 < 0.8  # default group: concurrent
