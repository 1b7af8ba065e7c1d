"""ray.util.actor_group.ActorGroup (reference: python/ray/util/tests/test_actor_group.py:
fan-out calls, metadata, add/remove, shutdown + restart, direct-call TypeError)."""
import pytest

import ray_community_amd as ray
from ray_community_amd.util.actor_group import ActorGroup


class Worker:
    def __init__(self, k=1):
        self.k = k

    def mul(self, x):
        return self.k * x


def test_actor_group_lifecycle():
    ray.init(num_cpus=4, log_to_driver=False)
    try:
        with pytest.warns(DeprecationWarning):
            g = ActorGroup(Worker, num_actors=3, init_args=(2,))
        assert len(g) == 3 and ray.get(g.mul.remote(5)) == [10, 10, 10]
        pids = {m.pid for m in g.actor_metadata}
        assert len(pids) == 3 and all(m.node_ip for m in g.actor_metadata)
        assert ray.get(g[1].actor.mul.remote(4)) == 8
        g.remove_actors([0, 2])
        assert len(g) == 1
        g.add_actors(2)
        assert ray.get(g.mul.remote(1)) == [2, 2, 2]
        with pytest.raises(TypeError):
            g.mul(1)
        g.shutdown()
        with pytest.raises(RuntimeError):
            g.mul
        g.start()
        assert ray.get(g.mul.remote(3)) == [6, 6, 6]
        g.shutdown(patience_s=0)
        with pytest.raises(ValueError):
            ActorGroup(Worker, num_actors=0)
    finally:
        ray.shutdown()
