"""Drives a worker group through one training run (reference:
``python/ray/train/_internal/backend_executor.py`` + ``train/trainer.py:TrainingIterator``)."""
from __future__ import annotations

import json
import logging
import os
import shutil
import time
from typing import Any, Callable, Dict, List, Optional

from ...exceptions import RayActorError, RayTaskError
from .._checkpoint import Checkpoint
from .session import TrainContext
from .worker_group import WorkerGroup

log = logging.getLogger("ray_community_amd.train")


class TrainingFailedError(RuntimeError):
    pass


class CheckpointManager:
    """Keeps the top-k persisted checkpoints (reference: ``train/_internal/checkpoint_manager.py``)."""

    def __init__(self, checkpoint_config):
        self.cfg = checkpoint_config
        self.entries: List[tuple] = []  # (checkpoint, metrics)
        self.latest: Optional[Checkpoint] = None

    def register(self, ckpt: Checkpoint, metrics: dict):
        self.latest = ckpt
        self.entries.append((ckpt, metrics))
        k = self.cfg.num_to_keep
        if k is None or len(self.entries) <= k:
            return
        attr = self.cfg.checkpoint_score_attribute
        if attr is None:
            victims = self.entries[:-k]
            keep = self.entries[-k:]
        else:
            sign = -1 if self.cfg.checkpoint_score_order == "max" else 1
            ranked = sorted(self.entries, key=lambda e: sign * float(e[1].get(attr, float("-inf") * -sign)))
            keep_set = {id(e) for e in ranked[:k]}
            # never delete the latest checkpoint (needed for fault tolerance)
            keep_set.add(id(self.entries[-1]))
            keep = [e for e in self.entries if id(e) in keep_set]
            victims = [e for e in self.entries if id(e) not in keep_set]
        for c, _ in victims:
            shutil.rmtree(c.path, ignore_errors=True)
        self.entries = keep

    @property
    def best_checkpoints(self):
        return list(self.entries)

    def best(self):
        attr = self.cfg.checkpoint_score_attribute
        if not self.entries:
            return None
        if attr is None:
            return self.entries[-1][0]
        f = max if self.cfg.checkpoint_score_order == "max" else min
        return f(self.entries, key=lambda e: e[1].get(attr, 0))[0]


def run_training(train_fn: Callable, config: Optional[dict], scaling_config, run_config, backend,
                 backend_config, datasets: Optional[dict], dataset_config, resume_from_checkpoint, trial_dir: str,
                 metadata: Optional[dict] = None, report_callback: Optional[Callable] = None,
                 experiment_name: str = ""):
    from ...air.result import Result

    os.makedirs(trial_dir, exist_ok=True)
    ckpt_mgr = CheckpointManager(run_config.checkpoint_config)
    latest = resume_from_checkpoint
    history: List[dict] = []
    failures = 0
    max_failures = run_config.failure_config.max_failures
    ckpt_index = 0
    last_metrics = None
    error = None
    while True:
        n = scaling_config.num_workers or 1
        wg = WorkerGroup(n, scaling_config._resources_per_worker_not_none, scaling_config.placement_strategy)
        try:
            infos = backend.on_start(wg, backend_config, scaling_config)
            shards = _split_datasets(datasets, n, dataset_config)
            from ..._private.worker import get

            starts = []
            for i, w in enumerate(wg.workers):
                ctx = TrainContext(world_rank=i, world_size=n, local_rank=infos[i]["local_rank"],
                                   local_world_size=infos[i]["local_world_size"], node_rank=infos[i]["node_rank"],
                                   experiment_name=experiment_name, trial_name=os.path.basename(trial_dir),
                                   trial_id=os.path.basename(trial_dir), trial_dir=trial_dir,
                                   storage_path=run_config.storage_path,
                                   metadata={**dict(metadata or {}), "_ckpt_start": ckpt_index})
                starts.append(w.start.remote(train_fn, config, ctx, latest, shards[i] if shards else {}))
            get(starts)
            done = [False] * n
            while not all(done):
                round_metrics = [None] * n
                round_ckpts = [None] * n
                got = [done[i] for i in range(n)]
                while not all(got):
                    for i, w in enumerate(wg.workers):
                        if got[i]:
                            continue
                        r = get(w.poll.remote(0.2))
                        if r[0] == "wait":
                            continue
                        got[i] = True
                        if r[0] == "result":
                            round_metrics[i] = r[1]
                            round_ckpts[i] = r[2]
                        elif r[0] == "done":
                            done[i] = True
                        elif r[0] == "error":
                            raise r[1]
                if all(m is None for m in round_metrics):
                    continue
                m = next(x for x in round_metrics if x is not None)
                m = dict(m)
                m.setdefault("timestamp", time.time())
                persisted = None
                paths = [c for c in round_ckpts if c is not None]
                if paths:
                    # workers already persisted into the trial dir (session.report)
                    dst = paths[0]
                    ckpt_index = max(ckpt_index, int(os.path.basename(dst).split("_")[-1]) + 1)
                    persisted = Checkpoint.from_directory(dst)
                    ckpt_mgr.register(persisted, m)
                    latest = persisted
                history.append(m)
                last_metrics = m
                with open(os.path.join(trial_dir, "result.json"), "a") as f:
                    f.write(json.dumps(_jsonable(m)) + "\n")
                if report_callback is not None:
                    stop = report_callback(m, persisted)
                    if stop:
                        done = [True] * n
            error = None
        except (RayTaskError, RayActorError, Exception) as e:  # noqa
            error = e
        finally:
            wg.shutdown()
        if error is None:
            break
        failures += 1
        if max_failures >= 0 and failures > max_failures:
            break
        log.warning("training failed (%s); restarting from %s (attempt %d)", type(error).__name__, latest, failures)
    err = None
    if error is not None:
        err = error if isinstance(error, TrainingFailedError) else TrainingFailedError(f"Training failed: {error}")
        err.__cause__ = error
    return Result(metrics=last_metrics, checkpoint=ckpt_mgr.latest or latest, error=err, path=trial_dir,
                  metrics_history=history, best_checkpoints=ckpt_mgr.best_checkpoints)


def _jsonable(d):
    out = {}
    for k, v in d.items():
        try:
            json.dumps(v)
            out[k] = v
        except TypeError:
            out[k] = repr(v)
    return out


def _split_datasets(datasets, n, dataset_config):
    if not datasets:
        return None
    shards = [dict() for _ in range(n)]
    for name, ds in datasets.items():
        split = True
        if dataset_config is not None and hasattr(dataset_config, "datasets_to_split"):
            dts = dataset_config.datasets_to_split
            split = dts == "all" or name in (dts or [])
        if split and hasattr(ds, "streaming_split"):
            parts = ds.streaming_split(n, equal=True)
            for i in range(n):
                shards[i][name] = parts[i]
        else:
            for i in range(n):
                shards[i][name] = ds.iterator() if hasattr(ds, "iterator") else ds
    return shards
