"""Compiled DAG behaviour (reference test models: python/ray/dag/tests/experimental/
test_accelerated_dag.py (several executions in flight with results read in order, numpy payloads,
fan-out to several actors, input kwargs))."""
import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd.dag import InputNode, MultiOutputNode


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


@ray.remote
class Worker:
    def __init__(self, k):
        self.k = k
        self.calls = 0

    def scale(self, x):
        self.calls += 1
        return x * self.k

    def num_calls(self):
        return self.calls


def test_executions_in_flight_read_in_order(session):
    w = Worker.remote(3)
    with InputNode() as inp:
        dag = w.scale.bind(inp)
    cd = dag.experimental_compile()
    try:
        refs = [cd.execute(i) for i in range(8)]          # submitted before any result is read
        assert [r.get(timeout=30) for r in refs] == [3 * i for i in range(8)]
    finally:
        cd.teardown()
    assert ray.get(w.num_calls.remote()) == 8


def test_numpy_payload_through_channels(session):
    a, b = Worker.remote(2), Worker.remote(-1)
    with InputNode() as inp:
        dag = b.scale.bind(a.scale.bind(inp))
    cd = dag.experimental_compile()
    try:
        x = np.arange(100_000, dtype=np.float32)
        out = cd.execute(x).get(timeout=30)
        assert isinstance(out, np.ndarray) and np.array_equal(out, -2 * x)
    finally:
        cd.teardown()


def test_fan_out_to_several_actors(session):
    ws = [Worker.remote(k) for k in (1, 2, 3, 4)]
    with InputNode() as inp:
        dag = MultiOutputNode([w.scale.bind(inp) for w in ws])
    cd = dag.experimental_compile()
    try:
        for v in (1, 5, 7):
            assert cd.execute(v).get(timeout=30) == [v, 2 * v, 3 * v, 4 * v]
    finally:
        cd.teardown()


def test_refs_read_out_of_order_and_buffer_cap(session):
    w = Worker.remote(5)
    with InputNode() as inp:
        dag = w.scale.bind(inp)
    cd = dag.experimental_compile(_max_buffered_results=3)
    try:
        r1, r2, r3 = cd.execute(1), cd.execute(2), cd.execute(3)
        assert r3.get(timeout=30) == 15                  # r1 and r2 move into the result buffer
        assert r1.get(timeout=30) == 5 and r2.get(timeout=30) == 10
        with pytest.raises(ValueError):
            r1.get(timeout=5)                            # each result is read once
        with pytest.raises(RuntimeError, match="max_buffered_results"):
            refs = [cd.execute(i) for i in range(6)]     # backed-up pipeline: too many unread results
            refs[-1].get(timeout=30)
    finally:
        cd.teardown()


@ray.remote
class Sleeper:
    def run(self, x):
        import time

        time.sleep(x)
        return x


def test_multi_output_timeout_then_retry_keeps_outputs_paired(session):
    """A get() that times out on the second output leaves the first output's channel released and
    its value kept: the retry returns this execution's outputs, and the next execution's after."""
    fast, slow = Worker.remote(1), Sleeper.remote()
    with InputNode() as inp:
        dag = MultiOutputNode([fast.scale.bind(inp), slow.run.bind(inp)])
    cd = dag.experimental_compile()
    try:
        r1 = cd.execute(1.5)
        with pytest.raises(Exception):
            r1.get(timeout=0.3)          # fast output read, the slow one times out
        assert r1.get(timeout=30) == [1.5, 1.5]
        assert cd.execute(0.1).get(timeout=30) == [0.1, 0.1]
    finally:
        cd.teardown()
