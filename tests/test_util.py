"""ray.util tests: ActorPool, Queue, multiprocessing Pool, collective (gloo), metrics, state, KV."""
import time

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd.util import collective as col


@ray.remote
class Doubler:
    def double(self, x):
        return 2 * x


def test_actor_pool(ray_start_regular):
    from ray_community_amd.util import ActorPool

    pool = ActorPool([Doubler.remote() for _ in range(3)])
    assert list(pool.map(lambda a, v: a.double.remote(v), range(10))) == [2 * i for i in range(10)]
    assert sorted(pool.map_unordered(lambda a, v: a.double.remote(v), range(10))) == [2 * i for i in range(10)]
    pool.submit(lambda a, v: a.double.remote(v), 4)
    assert pool.get_next() == 8
    assert not pool.has_next()


def test_actor_pool_backlog_ordering_and_membership(ray_start_regular):
    from ray_community_amd.util import ActorPool

    @ray.remote
    class Sleeper:
        def run(self, x):
            time.sleep(0.3 if x == 0 else 0.01)
            return x

    a, b = Sleeper.remote(), Sleeper.remote()
    pool = ActorPool([a, b])
    for v in range(5):  # 2 run, 3 wait in the backlog for an idle actor
        pool.submit(lambda act, v: act.run.remote(v), v)
    assert not pool.has_free() and pool.pop_idle() is None
    first = pool.get_next_unordered()
    assert first != 0  # item 0 is the slow one
    rest = [pool.get_next() for _ in range(4)]  # ordered retrieval skips the ticket already taken
    assert sorted([first] + rest) == list(range(5)) and rest == sorted(rest)
    assert pool.has_free()
    idle = pool.pop_idle()
    assert idle is not None
    other = b if idle is a else a
    with pytest.raises(ValueError):
        pool.push(other)  # still a member of the pool
    pool.push(idle)
    with pytest.raises(StopIteration):
        pool.get_next()
    pool.submit(lambda act, v: act.run.remote(v), 0)
    with pytest.raises(TimeoutError):
        pool.get_next(timeout=0.01)


def test_queue_bounded_blocking_and_async(ray_start_regular):
    from ray_community_amd.util.queue import Empty, Full, Queue

    q = Queue(maxsize=2)
    q.put(1)
    q.put(2)
    assert q.full() and len(q) == 2
    with pytest.raises(Full):
        q.put(3, block=False)
    with pytest.raises(Full):
        q.put(3, timeout=0.1)
    with pytest.raises(Full):
        q.put_nowait_batch([3, 4])

    @ray.remote
    def late_consumer(q):
        time.sleep(0.3)
        return q.get()

    r = late_consumer.remote(q)
    q.put(3, timeout=10)  # blocks until the consumer frees a slot
    assert ray.get(r) == 1 and q.get_nowait_batch(2) == [2, 3]
    with pytest.raises(Empty):
        q.get_nowait_batch(1)

    @ray.remote
    class User:
        async def roundtrip(self, q):
            await q.put_async("x")
            return await q.get_async(timeout=5)

    assert ray.get(User.remote().roundtrip.remote(q)) == "x"
    q.shutdown()


def test_queue(ray_start_regular):
    from ray_community_amd.util.queue import Empty, Queue

    q = Queue(maxsize=10)
    for i in range(5):
        q.put(i)
    assert q.qsize() == 5
    assert [q.get() for _ in range(5)] == list(range(5))
    assert q.empty()
    with pytest.raises(Empty):
        q.get(block=False)
    with pytest.raises(Empty):
        q.get(timeout=0.1)

    @ray.remote
    def producer(q):
        for i in range(3):
            q.put(i)

    ray.get(producer.remote(q))
    assert q.get_nowait_batch(3) == [0, 1, 2]


def test_multiprocessing_pool(ray_start_regular):
    from ray_community_amd.util.multiprocessing import Pool

    with Pool(processes=2) as p:
        assert p.map(abs, [-1, -2, 3]) == [1, 2, 3]
        assert p.starmap(pow, [(2, 3), (3, 2)]) == [8, 9]
        assert p.apply(max, (1, 5)) == 5
        assert sorted(p.imap_unordered(abs, [-3, -4])) == [3, 4]


def test_collective_gloo_actors(ray_start_regular):
    @ray.remote
    class W:
        def __init__(self, rank):
            self.rank = rank

        def setup(self, world):
            col.init_collective_group(world, self.rank, backend="gloo", group_name="g")
            return True

        def run(self):
            import torch

            t = torch.ones(4) * (self.rank + 1)
            col.allreduce(t, group_name="g")
            b = torch.full((2,), float(self.rank))
            col.broadcast(b, src_rank=1, group_name="g")
            outs = [torch.zeros(3) for _ in range(2)]
            col.allgather(outs, torch.full((3,), float(self.rank)), group_name="g")
            if self.rank == 0:
                col.send(torch.arange(3.0), 1, group_name="g")
                got = None
            else:
                got = torch.zeros(3)
                col.recv(got, 0, group_name="g")
                got = got.tolist()
            rs = torch.zeros(2)
            col.reducescatter(rs, [torch.ones(2) * (self.rank + 1), torch.ones(2) * 10], group_name="g")
            col.barrier(group_name="g")
            return t.tolist(), b.tolist(), [o.tolist() for o in outs], got, rs.tolist(), col.get_rank("g")

    ws = [W.remote(i) for i in range(2)]
    assert ray.get([w.setup.remote(2) for w in ws]) == [True, True]
    r0, r1 = ray.get([w.run.remote() for w in ws])
    assert r0[0] == [3.0] * 4 and r1[0] == [3.0] * 4
    assert r0[1] == [1.0, 1.0]
    assert r1[2] == [[0.0] * 3, [1.0] * 3]
    assert r1[3] == [0.0, 1.0, 2.0]
    assert r0[4] == [3.0, 3.0] and r1[4] == [20.0, 20.0]
    assert (r0[5], r1[5]) == (0, 1)


def test_collective_multigpu_list_forms_gloo(ray_start_regular):
    """*_multigpu with two local tensors per rank (one-GPU-per-process design: local combine, one
    collective, copy back) match the reference's per-GPU semantics."""
    @ray.remote
    class W:
        def __init__(self, rank):
            self.rank = rank

        def run(self, world):
            import torch

            col.init_collective_group(world, self.rank, backend="gloo", group_name="mg")
            r = self.rank
            ts = [torch.full((2,), float(r + 1)), torch.full((2,), float(10 * (r + 1)))]
            col.allreduce_multigpu(ts, group_name="mg")
            red = [torch.full((1,), float(r + 1)), torch.full((1,), 1.0)]
            col.reduce_multigpu(red, dst_rank=1, dst_tensor=1, group_name="mg")
            bc = [torch.full((1,), float(r)), torch.full((1,), float(100 + r))]
            col.broadcast_multigpu(bc, src_rank=0, src_tensor=1, group_name="mg")
            outs = [[torch.zeros(1) for _ in range(world * 2)] for _ in range(2)]
            col.allgather_multigpu(outs, [torch.full((1,), float(10 * r)), torch.full((1,), float(10 * r + 1))],
                                   group_name="mg")
            ins = [[torch.full((1,), float(k)) for k in range(world * 2)] for _ in range(2)]
            rs = [torch.zeros(1), torch.zeros(1)]
            col.reducescatter_multigpu(rs, ins, group_name="mg")
            return ([t.tolist() for t in ts], red[1].item(), [b.item() for b in bc],
                    [o.item() for o in outs[1]], [x.item() for x in rs], col.gloo_available())

    ws = [W.remote(i) for i in range(2)]
    r0, r1 = ray.get([w.run.remote(2) for w in ws])
    assert r0[0] == [[33.0, 33.0], [33.0, 33.0]] and r1[0] == r0[0]  # (1+10) + (2+20)
    assert r1[1] == 1 + 1 + 2 + 1  # sum over both ranks' local lists, landed in tensor 1 of rank 1
    assert r0[2] == [100.0, 100.0] and r1[2] == [100.0, 100.0]
    assert r1[3] == [0.0, 1.0, 10.0, 11.0]
    assert r0[4] == [0.0, 4.0] and r1[4] == [8.0, 12.0]  # 2 local lists x 2 ranks x k
    assert r0[5] is True


def test_collective_declarative(ray_start_regular):
    @ray.remote
    class W:
        def go(self):
            import torch

            t = torch.ones(2)
            col.allreduce(t, group_name="decl")
            return t.tolist()

    ws = [W.remote() for _ in range(3)]
    col.create_collective_group(ws, 3, [0, 1, 2], backend="gloo", group_name="decl")
    assert ray.get([w.go.remote() for w in ws]) == [[3.0, 3.0]] * 3


def test_metrics():
    from ray_community_amd.util.metrics import Counter, Gauge, Histogram, export_prometheus

    c = Counter("reqs", "requests", tag_keys=("route",))
    c.inc(2, {"route": "/a"})
    g = Gauge("temp")
    g.set(3.5)
    h = Histogram("lat", boundaries=[1, 10], tag_keys=("x",)).set_default_tags({"x": "y"})
    h.observe(5)
    txt = export_prometheus()
    assert 'reqs{route="/a"} 2.0' in txt and "temp 3.5" in txt and 'lat_bucket{x="y",le="10"} 1' in txt
    with pytest.raises(ValueError):
        c.inc(1, {"bad": 1})


def test_state_api_and_kv(ray_start_regular):
    from ray_community_amd.experimental import internal_kv as kv
    from ray_community_amd.util import state

    @ray.remote
    def f():
        return 1

    ray.get([f.remote() for _ in range(3)])
    a = Doubler.remote()
    ray.get(a.double.remote(1))
    tasks = state.list_tasks()
    assert sum(1 for t in tasks if t["state"] == "FINISHED") >= 3
    assert any(x["class_name"] == "Doubler" and x["state"] == "ALIVE" for x in state.list_actors())
    assert state.summarize_tasks()["cluster"]["total_tasks"] >= 4
    assert len(state.list_nodes()) == 1
    assert not kv._internal_kv_put("k", b"v")
    assert kv._internal_kv_get("k") == b"v"
    assert kv._internal_kv_list("k") == [b"k"]
    assert kv._internal_kv_del("k") == 1
    tl = ray.timeline()
    assert any(e["name"] == "f" for e in tl)
