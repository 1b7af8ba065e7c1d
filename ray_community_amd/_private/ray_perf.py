"""Core-runtime microbenchmark (the ``ray microbenchmark`` suite).

Same workloads and the same names as the reference suite (reference:
``python/ray/_private/ray_perf.py:93-330``, timing harness
``python/ray/_private/ray_microbenchmark_helpers.py:15-47``) so results line up row by row with
``release/release_logs/2.9.3/microbenchmark.json``; the timing windows are shorter (``--quick``
shrinks them further for CI). Reported as ops/s (GB/s for the gigabyte rows).

Two driver placements (``mode``):

* ``colocated``: ``ray.init()`` starts the head inside the benchmark process (the default of
  ``ray.init`` here), so driver -> head calls are in-process calls under the head's lock;
* ``separate``: a head started by ``python -m ray_community_amd start --head`` in its own
  process, the benchmark connecting with ``ray.init(address="auto")`` like the reference's
  ``ray microbenchmark`` driver does: every control call crosses a Unix socket.

In both modes ``ray.put`` of an object <= 100 KB is stored inline in the owner (this process),
not in the shared-memory store, so the two "Plasma Store" put/get rows measure the owner's
in-process store; the extra ``(shm store, 128 KB)`` rows put / get objects just above the inline
threshold, which go through the native shm store (no reference row).
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import multiprocessing
import os
import subprocess
import sys
import tempfile
import time
from typing import Callable, List, Optional, Tuple

import numpy as np

import ray_community_amd as ray

# reference numbers: release/release_logs/2.9.3/microbenchmark.json (m5.16xlarge, 64 vCPU)
REFERENCE = {
    "single_client_get_calls_Plasma_Store": 10181.63,
    "single_client_put_calls_Plasma_Store": 5544.98,
    "multi_client_put_calls_Plasma_Store": 12676.96,
    "single_client_put_gigabytes": 20.88,
    "single_client_tasks_and_get_batch": 8.48,
    "multi_client_put_gigabytes": 35.88,
    "single_client_get_object_containing_10k_refs": 12.39,
    "single_client_wait_1k_refs": 5.49,
    "single_client_tasks_sync": 1006.89,
    "single_client_tasks_async": 8443.54,
    "multi_client_tasks_async": 25165.64,
    "1_1_actor_calls_sync": 2033.2,
    "1_1_actor_calls_async": 8886.33,
    "1_1_actor_calls_concurrent": 5094.68,
    "1_n_actor_calls_async": 8569.98,
    "n_n_actor_calls_async": 27666.56,
    "n_n_actor_calls_with_arg_async": 2829.27,
    "1_1_async_actor_calls_sync": 1291.65,
    "1_1_async_actor_calls_async": 3433.73,
    "1_1_async_actor_calls_with_args_async": 2307.18,
    "1_n_async_actor_calls_async": 7455.79,
    "n_n_async_actor_calls_async": 22927.08,
    "placement_group_create/removal": 796.6,
}


def _key(name: str) -> str:
    return name.replace(" ", "_").replace(":", "_").replace("-", "_").replace("(", "").replace(")", "")


class _Timer:
    def __init__(self, window: float, rounds: int, pattern: str = ""):
        self.window = window
        self.rounds = rounds
        self.pattern = pattern
        self.results: List[Tuple[str, float, float]] = []

    def __call__(self, name: str, fn: Callable[[], object], multiplier: float = 1.0):
        if self.pattern and self.pattern not in name:
            return
        start = time.perf_counter()
        count = 0
        while time.perf_counter() - start < self.window / 2:  # warmup
            fn()
            count += 1
        step = count // 10 + 1
        stats = []
        for _ in range(self.rounds):
            start = time.perf_counter()
            count = 0
            while time.perf_counter() - start < self.window:
                for _ in range(step):
                    fn()
                count += step
            stats.append(multiplier * count / (time.perf_counter() - start))
        mean, sd = float(np.mean(stats)), float(np.std(stats))
        print(f"{name} per second {mean:.2f} +- {sd:.2f}", flush=True)
        self.results.append((name, mean, sd))


@ray.remote(num_cpus=0)
class Actor:
    def small_value(self):
        return b"ok"

    def small_value_arg(self, x):
        return b"ok"

    def small_value_batch(self, n):
        ray.get([small_value.remote() for _ in range(n)])


@ray.remote(num_cpus=0)
class AsyncActor:
    async def small_value(self):
        return b"ok"

    async def small_value_with_arg(self, x):
        return b"ok"

    async def small_value_batch(self, n):
        await asyncio.wait([small_value.remote() for _ in range(n)])


@ray.remote(num_cpus=0)
class Client:
    def __init__(self, servers):
        self.servers = servers if isinstance(servers, list) else [servers]

    def small_value_batch(self, n):
        results = []
        for s in self.servers:
            results.extend([s.small_value.remote() for _ in range(n)])
        ray.get(results)

    def small_value_batch_arg(self, n):
        x = ray.put(0)
        results = []
        for s in self.servers:
            results.extend([s.small_value_arg.remote(x) for _ in range(n)])
        ray.get(results)


@ray.remote
def small_value():
    return b"ok"


@ray.remote
def create_object_containing_ref():
    obj_refs = []
    for _ in range(10000):
        obj_refs.append(ray.put(1))
    return obj_refs


@contextlib.contextmanager
def _session(mode: str, ncpu: int, resources: Optional[dict] = None):
    if mode == "colocated":
        ray.init(num_cpus=ncpu, resources=resources, log_to_driver=False)
        try:
            yield
        finally:
            ray.shutdown()
        return
    if mode != "separate":
        raise ValueError(f"mode must be 'colocated' or 'separate', not {mode!r}")
    tmp = tempfile.mkdtemp(prefix="rca_perf_")
    prev = os.environ.get("RCA_TEMP_DIR")
    env = dict(os.environ, RCA_TEMP_DIR=tmp)
    cli = [sys.executable, "-m", "ray_community_amd"]
    args = ["start", "--head", "--num-cpus", str(ncpu)] + (["--resources", json.dumps(resources)] if resources else [])
    r = subprocess.run(cli + args, env=env, capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        raise RuntimeError(f"head start failed: {r.stderr[-2000:]}")
    os.environ["RCA_TEMP_DIR"] = tmp
    try:
        ray.init(address="auto", log_to_driver=False)
        try:
            yield
        finally:
            ray.shutdown()
    finally:
        subprocess.run(cli + ["stop", "--force"], env=env, capture_output=True, text=True, timeout=120)
        if prev is None:
            os.environ.pop("RCA_TEMP_DIR", None)
        else:
            os.environ["RCA_TEMP_DIR"] = prev


def run(window: float = 2.0, rounds: int = 4, pattern: str = "", scale: float = 1.0,
        mode: str = "colocated") -> List[Tuple[str, float, float]]:
    """Run the suite. ``scale`` < 1 shrinks batch sizes (CI); the ops/s definition is unchanged.
    ``mode``: ``colocated`` (head in this process) or ``separate`` (head in its own process)."""
    t = _Timer(window, rounds, pattern)
    ncpu = max(2, multiprocessing.cpu_count())
    with _session(mode, ncpu):
        value = ray.put(0)
        t("single client get calls (Plasma Store)", lambda: ray.get(value))
        t("single client put calls (Plasma Store)", lambda: ray.put(0))
        big = np.zeros(128 * 1024 // 8, dtype=np.int64)  # above the 100 KB inline threshold
        shm_value = ray.put(big)
        t("single client get calls (shm store, 128 KB)", lambda: ray.get(shm_value))
        t("single client put calls (shm store, 128 KB)", lambda: ray.put(big))
        del shm_value

        @ray.remote
        def do_put_small():
            for _ in range(100):
                ray.put(0)

        t("multi client put calls (Plasma Store)", lambda: ray.get([do_put_small.remote() for _ in range(10)]), 1000)

        arr = np.zeros(int(100 * 1024 * 1024 * scale), dtype=np.int64)
        t("single client put gigabytes", lambda: ray.put(arr), 8 * 0.1 * scale)

        nb = max(10, int(1000 * scale))
        t("single client tasks and get batch", lambda: ray.get([small_value.remote() for _ in range(nb)]))

        @ray.remote
        def do_put():
            for _ in range(10):
                ray.put(np.zeros(int(10 * 1024 * 1024 * scale), dtype=np.int64))

        t("multi client put gigabytes", lambda: ray.get([do_put.remote() for _ in range(10)]), 10 * 8 * 0.1 * scale)

        obj_containing_ref = create_object_containing_ref.remote()
        ray.get(obj_containing_ref)
        t("single client get object containing 10k refs", lambda: ray.get(obj_containing_ref))

        def wait_multiple_refs():
            not_ready = [small_value.remote() for _ in range(nb)]
            for _ in range(nb):
                _ready, not_ready = ray.wait(not_ready)

        t("single client wait 1k refs", wait_multiple_refs)
        t("single client tasks sync", lambda: ray.get(small_value.remote()))
        t("single client tasks async", lambda: ray.get([small_value.remote() for _ in range(nb)]), nb)

        n, m = max(100, int(10000 * scale)), 4
        actors = [Actor.remote() for _ in range(m)]
        t("multi client tasks async", lambda: ray.get([a.small_value_batch.remote(n) for a in actors]), n * m)

        a = Actor.remote()
        t("1:1 actor calls sync", lambda: ray.get(a.small_value.remote()))
        a = Actor.remote()
        t("1:1 actor calls async", lambda: ray.get([a.small_value.remote() for _ in range(nb)]), nb)
        a = Actor.options(max_concurrency=16).remote()
        t("1:1 actor calls concurrent", lambda: ray.get([a.small_value.remote() for _ in range(nb)]), nb)

        n = max(100, int(5000 * scale))
        n_half = max(1, ncpu // 2)
        actors = [Actor.remote() for _ in range(n_half)]
        client = Client.remote(actors)
        t("1:n actor calls async", lambda: ray.get(client.small_value_batch.remote(n)), n * len(actors))

        a = [Actor.remote() for _ in range(n_half)]

        @ray.remote
        def work(actors):
            ray.get([actors[i % n_half].small_value.remote() for i in range(n)])

        t("n:n actor calls async", lambda: ray.get([work.remote(a) for _ in range(m)]), m * n)

        n = max(50, int(1000 * scale))
        actors = [Actor.remote() for _ in range(n_half)]
        clients = [Client.remote(x) for x in actors]
        t("n:n actor calls with arg async", lambda: ray.get([c.small_value_batch_arg.remote(n) for c in clients]),
          n * len(clients))

        aa = AsyncActor.remote()
        t("1:1 async-actor calls sync", lambda: ray.get(aa.small_value.remote()))
        aa = AsyncActor.remote()
        t("1:1 async-actor calls async", lambda: ray.get([aa.small_value.remote() for _ in range(nb)]), nb)
        aa = AsyncActor.remote()
        t("1:1 async-actor calls with args async",
          lambda: ray.get([aa.small_value_with_arg.remote(i) for i in range(nb)]), nb)

        n = max(100, int(5000 * scale))
        actors = [AsyncActor.remote() for _ in range(n_half)]
        client = Client.remote(actors)
        t("1:n async-actor calls async", lambda: ray.get(client.small_value_batch.remote(n)), n * len(actors))

        a = [AsyncActor.remote() for _ in range(n_half)]

        @ray.remote
        def async_actor_work(actors):
            ray.get([actors[i % n_half].small_value.remote() for i in range(n)])

        t("n:n async-actor calls async", lambda: ray.get([async_actor_work.remote(a) for _ in range(m)]), m * n)

    with _session(mode, ncpu, {"custom": 100}):
        from ..util.placement_group import placement_group, remove_placement_group

        npg = 100

        def pg_create_removal():
            pgs = [placement_group([{"custom": 0.001}]) for _ in range(npg)]
            for pg in pgs:
                pg.wait(timeout_seconds=30)
            for pg in pgs:
                remove_placement_group(pg)

        t("placement group create/removal", pg_create_removal, npg)
    return t.results


def report(results, out: Optional[str] = None, mode: str = "colocated") -> dict:
    rows = {}
    for name, mean, sd in results:
        k = _key(name)
        ref = REFERENCE.get(k)
        rows[k] = {"value": round(mean, 2), "sd": round(sd, 2), "reference": ref,
                   "vs_reference": round(mean / ref, 3) if ref else None}
    doc = {"suite": "core_microbenchmark", "mode": mode, "cpus": multiprocessing.cpu_count(),
           "reference_hw": "m5.16xlarge (64 vCPU)", "results": rows}
    if out:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as f:
            json.dump(doc, f, indent=1)
    return doc
