"""ray:// remote drivers (util/client; reference: python/ray/util/client/, tests
python/ray/tests/test_client*.py): a head started by the CLI with --ray-client-server-port,
driven from this process over TCP."""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

import ray_community_amd as ray

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def client_head(tmp_path):
    port = _free_port()
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    env.pop("RAY_ADDRESS", None)
    cmd = [sys.executable, "-m", "ray_community_amd", "start", "--head", "--block", "--num-cpus", "4",
           "--temp-dir", str(tmp_path), "--ray-client-server-port", str(port)]
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    deadline = time.time() + 120
    while time.time() < deadline:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=1).close()
            break
        except OSError:
            if proc.poll() is not None:
                raise RuntimeError(proc.stdout.read().decode())
            time.sleep(0.2)
    yield f"ray://127.0.0.1:{port}"
    proc.terminate()
    try:
        proc.wait(timeout=30)
    except subprocess.TimeoutExpired:
        proc.kill()


@ray.remote
def _square(x):
    return x * x


@ray.remote
def _total(arr):
    return float(arr.sum())


@ray.remote
class _Counter:
    def __init__(self, start=0):
        self.n = start

    def incr(self, k=1):
        self.n += k
        return self.n

    def big(self, n):
        return np.arange(n, dtype=np.float64)


def test_remote_driver_tasks_objects_actors(client_head):
    ray.init(client_head)
    try:
        from ray_community_amd.util.client import is_connected

        assert is_connected()
        assert ray.get([_square.remote(i) for i in range(10)]) == [i * i for i in range(10)]
        # large objects both ways: put (written into the node's shm by the server) and results
        big = np.random.default_rng(0).random(400_000)  # 3.2 MB
        ref = ray.put(big)
        assert np.array_equal(ray.get(ref), big)
        assert ray.get(_total.remote(ref)) == pytest.approx(float(big.sum()))
        assert ray.get(_total.remote(big)) == pytest.approx(float(big.sum()))  # by-value arg
        # chained refs and wait
        refs = [_square.remote(_square.remote(i)) for i in range(5)]
        ready, rest = ray.wait(refs, num_returns=5, timeout=60)
        assert len(ready) == 5 and not rest
        assert ray.get(refs) == [i ** 4 for i in range(5)]
        # actors: ordered calls, named lookup, large returns, kill
        c = _Counter.options(name="ctr", namespace="cli").remote(10)
        assert ray.get([c.incr.remote() for _ in range(5)]) == [11, 12, 13, 14, 15]
        c2 = ray.get_actor("ctr", namespace="cli")
        assert ray.get(c2.incr.remote(5)) == 20
        arr = ray.get(c.big.remote(300_000))
        assert arr.shape == (300_000,) and arr[-1] == 299_999
        ray.kill(c)
        with pytest.raises(ray.exceptions.RayActorError):
            ray.get(c.incr.remote(), timeout=60)
        assert ray.cluster_resources().get("CPU") == 4
        # task errors surface with their cause
        @ray.remote
        def boom():
            raise ValueError("bad")

        with pytest.raises(ValueError):
            ray.get(boom.remote())
    finally:
        ray.shutdown()
    # a second remote driver after the first one left
    ray.init(client_head)
    try:
        assert ray.get(_square.remote(7)) == 49
    finally:
        ray.shutdown()


def test_parse_address():
    from ray_community_amd.util.client import parse_address

    assert parse_address("ray://10.0.0.1:12345") == ("10.0.0.1", 12345)
    assert parse_address("ray://headnode") == ("headnode", 10001)


def test_util_client_connect_and_disconnect(client_head):
    """ray.util.client_connect.connect / disconnect (reference util/client_connect.py)."""
    from ray_community_amd.util.client_connect import connect, disconnect

    info = connect(client_head[len("ray://"):], namespace="cc")
    try:
        assert info["address"] == client_head

        @ray.remote
        def f(x):
            return x + 1

        assert ray.get(f.remote(1)) == 2
        with pytest.raises(RuntimeError):
            connect(client_head)
        assert connect(client_head, ray_init_kwargs={"ignore_reinit_error": True})["reused"]
    finally:
        disconnect()
    assert not ray.is_initialized()
    disconnect()  # idempotent
