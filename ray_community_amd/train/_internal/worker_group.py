"""Training worker group (reference: ``python/ray/train/_internal/worker_group.py``).

One actor per worker, all placed in ONE placement group (one bundle per worker, PACK by
default) so a DDP group lands on as few nodes as possible — on an MI355X node that means all
ranks share the xGMI fabric.
"""
from __future__ import annotations

import os
import queue
import socket
import threading
import time
import traceback
from typing import Any, Callable, Dict, List, Optional


class _TrainWorker:
    """Actor body for one training worker."""

    def __init__(self):
        self._thread = None
        self._result_q: "queue.Queue" = queue.Queue()
        self._done = False
        self._error = None
        self._ret = None

    def node_info(self):
        import ray_community_amd as ray

        ctx = ray.get_runtime_context()
        vis = os.environ.get("HIP_VISIBLE_DEVICES", "")
        return {"node_id": ctx.get_node_id(), "pid": os.getpid(), "gpu_ids": ray.get_gpu_ids(),
                "visible": [v for v in vis.split(",") if v != ""], "hostname": socket.gethostname()}

    def set_env(self, env: Dict[str, str]):
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        return True

    def free_port(self):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    def execute(self, fn, *args, **kwargs):
        return fn(*args, **kwargs)

    def idle(self) -> bool:
        """No training thread running (a finished trial's actor can take the next one)."""
        return self._thread is None or not self._thread.is_alive()

    def start(self, fn, config, context, checkpoint, dataset_shards):
        from . import session as S

        self._done, self._error, self._ret = False, None, None

        sess = S.init_session(context, checkpoint=checkpoint, dataset_shards=dataset_shards)
        self._sess = sess

        def run():
            try:
                if config is None:
                    self._ret = fn()
                else:
                    self._ret = fn(config)
            except BaseException as e:  # noqa
                self._error = e
                self._tb = traceback.format_exc()
            finally:
                self._done = True
                sess.results.put(None)

        self._thread = threading.Thread(target=run, name="rca-train-loop", daemon=True)
        self._thread.start()
        return True

    def poll(self, timeout: float = 1.0):
        """Return ("result", metrics, checkpoint_path) | ("done", return_value) | ("error", exc) | ("wait",)."""
        sess = getattr(self, "_sess", None)
        if sess is None:  # threaded actor: a poll can overtake start()
            time.sleep(min(timeout, 0.05))
            return ("wait",)
        try:
            item = sess.results.get(timeout=timeout)
        except queue.Empty:
            return ("wait",)
        if item is None:
            if self._error is not None:
                from ...exceptions import RayTaskError

                return ("error", RayTaskError.from_exception(self._error, "train_loop_per_worker"))
            return ("done", self._ret)
        metrics, ckpt = item
        return ("result", metrics, ckpt.path if ckpt is not None else None)

    def shutdown(self):
        try:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass
        return True


class WorkerGroup:
    def __init__(self, num_workers: int, resources_per_worker: Dict[str, float], placement_strategy: str = "PACK",
                 actor_cls=None):
        from ...actor import ActorClass
        from ...util.placement_group import placement_group
        from ...util.scheduling_strategies import PlacementGroupSchedulingStrategy

        self.num_workers = num_workers
        res = dict(resources_per_worker)
        self.pg = placement_group([dict(res) for _ in range(num_workers)], strategy=placement_strategy)
        from ..._private.worker import get

        get(self.pg.ready(), timeout=None)
        opts = {"num_cpus": res.pop("CPU", 0), "num_gpus": res.pop("GPU", 0), "resources": res or None,
                "max_concurrency": 4}
        cls = ActorClass(actor_cls or _TrainWorker, {k: v for k, v in opts.items() if v is not None})
        self.workers = [cls.options(scheduling_strategy=PlacementGroupSchedulingStrategy(self.pg, i)).remote()
                        for i in range(num_workers)]

    def execute(self, fn, *args, **kwargs):
        from ..._private.worker import get

        return get([w.execute.remote(fn, *args, **kwargs) for w in self.workers])

    def execute_single(self, idx, fn, *args, **kwargs):
        from ..._private.worker import get

        return get(self.workers[idx].execute.remote(fn, *args, **kwargs))

    def shutdown(self):
        from ..._private.worker import get, kill
        from ...util.placement_group import remove_placement_group

        try:
            get([w.shutdown.remote() for w in self.workers], timeout=10)
        except Exception:
            pass
        for w in self.workers:
            try:
                kill(w)
            except Exception:
                pass
        try:
            remove_placement_group(self.pg)
        except Exception:
            pass
        self.workers = []

    def __len__(self):
        return len(self.workers)
