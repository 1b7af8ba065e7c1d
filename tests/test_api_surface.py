"""Top-level / util API surface that users reach for (reference python/ray/__init__.py and
python/ray/util/__init__.py __all__): client builder, Language and cross-language stubs,
show_in_dashboard, list_named_actors, accelerators, log_once, serializers, remote pdb."""
import socket
import threading
import time

import pytest

import ray_community_amd as ray
from ray_community_amd.util import state


def test_reference_exports_present():
    import ray_community_amd.util as u

    for n in ["client", "ClientBuilder", "Language", "java_function", "java_actor_class", "cpp_function",
              "show_in_dashboard"]:
        assert hasattr(ray, n), n
    for n in ["accelerators", "disable_log_once_globally", "enable_periodic_logging", "log_once", "pdb", "connect",
              "disconnect", "register_serializer", "deregister_serializer", "list_named_actors"]:
        assert hasattr(u, n), n
    assert u.accelerators.AMD_INSTINCT_MI355X == "AMD-Instinct-MI355X"
    with pytest.raises(NotImplementedError):
        ray.java_function("Cls", "f")


def test_list_named_actors_and_show_in_dashboard(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False, namespace="ns1")

    @ray.remote
    class A:
        def note(self, m):
            ray.show_in_dashboard(m)
            return True

    a = A.options(name="alpha").remote()
    b = A.options(name="beta", namespace="other").remote()
    ray.get([a.note.remote("warming up"), b.note.remote("x")])
    assert ray.util.list_named_actors() == ["alpha"]
    allns = ray.util.list_named_actors(all_namespaces=True)
    assert {"name": "beta", "namespace": "other"} in allns and {"name": "alpha", "namespace": "ns1"} in allns
    row = state.list_actors(filters=[("name", "=", "alpha")])[0]
    assert row["annotations"] == {"message": "warming up"}


def test_log_once_and_serializer_registration(shutdown_only):
    from ray_community_amd.util import debug

    debug.enable_periodic_logging()
    assert ray.util.log_once("k1") and not ray.util.log_once("k1")

    class Point:
        def __init__(self, x):
            self.x = x

    ray.init(num_cpus=1, include_dashboard=False, log_to_driver=False)
    ray.util.register_serializer(Point, serializer=lambda p: p.x * 10, deserializer=lambda v: Point(v + 1))
    assert ray.get(ray.put(Point(2))).x == 21
    ray.util.deregister_serializer(Point)


def test_remote_pdb_session_in_a_task(shutdown_only, tmp_path):
    """A task hits set_trace(); a TCP client drives pdb (prints a local, continues) and the task
    finishes with the value computed after the breakpoint."""
    ray.init(num_cpus=1, include_dashboard=False, log_to_driver=False)
    port_holder = socket.socket()
    port_holder.bind(("127.0.0.1", 0))
    port = port_holder.getsockname()[1]
    port_holder.close()

    @ray.remote
    def buggy(v):
        from ray_community_amd.util import pdb

        secret = v * 7
        pdb.set_trace(port=port, timeout=60)
        return secret + 1

    ref = buggy.remote(6)
    deadline = time.time() + 30
    conn = None
    while time.time() < deadline:
        try:
            conn = socket.create_connection(("127.0.0.1", port), timeout=5)
            break
        except OSError:
            time.sleep(0.1)
    assert conn is not None
    f = conn.makefile("rw")
    got = []

    def reader():
        try:
            for line in f:
                got.append(line)
        except Exception:  # noqa
            pass

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    f.write("p secret\n")
    f.flush()
    time.sleep(0.5)
    f.write("c\n")
    f.flush()
    assert ray.get(ref, timeout=30) == 43
    assert any("42" in ln for ln in got)
    conn.close()
