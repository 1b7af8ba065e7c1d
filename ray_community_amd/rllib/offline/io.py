"""Offline input / output plumbing of the old API stack (reference: rllib/offline/
{input_reader,output_writer,mixed_input,shuffled_input,dataset_writer,d4rl_reader,
feature_importance}.py, offline/__init__.py:get_offline_io_resource_bundles)."""
from __future__ import annotations

import random
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np

from ..env.policy_server_input import IOContext
from ..policy.sample_batch import SampleBatch, concat_samples


class InputReader:
    """Produces experience batches: implement ``next()``."""

    def next(self) -> SampleBatch:
        raise NotImplementedError

    def __iter__(self):
        while True:
            yield self.next()


class OutputWriter:
    def write(self, sample_batch: SampleBatch) -> None:
        raise NotImplementedError


class NoopOutput(OutputWriter):
    def write(self, sample_batch):
        pass


def _reader(spec, ioctx: IOContext) -> InputReader:
    from . import JsonReader

    if spec == "sampler":
        return _SamplerInput(ioctx.worker)
    if isinstance(spec, str):
        return _Adapt(JsonReader(spec))
    if callable(spec):
        return spec(ioctx)
    return spec


class _Adapt(InputReader):
    def __init__(self, reader):
        self.reader = reader

    def next(self):
        return self.reader.next()


class _SamplerInput(InputReader):
    def __init__(self, runner):
        if runner is None:
            raise ValueError("'sampler' input needs IOContext.worker (an env runner)")
        self.runner = runner

    def next(self):
        return self.runner.sample()


class MixedInput(InputReader):
    """Mixes sources by probability: ``{"sampler": 0.4, "/tmp/data": 0.6}`` (a source is
    "sampler", a JSON path / glob, a reader factory ``f(ioctx)`` or an InputReader)."""

    def __init__(self, dist: Dict[Any, float], ioctx: IOContext, seed: Optional[int] = None):
        total = float(sum(dist.values()))
        if abs(total - 1.0) > 1e-4:
            raise ValueError(f"MixedInput probabilities must sum to 1, got {total}")
        self.choices = [_reader(k, ioctx) for k in dist]
        self.p = [float(v) for v in dist.values()]
        self._rng = np.random.default_rng(seed)

    def next(self) -> SampleBatch:
        return self.choices[int(self._rng.choice(len(self.choices), p=self.p))].next()


class ShuffledInput(InputReader):
    """Keeps ``n`` batches and hands out a random one, refilling from ``child`` (n <= 1: pass-through)."""

    def __init__(self, child: InputReader, n: int = 0, seed: Optional[int] = None):
        self.child = child
        self.n = int(n)
        self.buffer: List[SampleBatch] = []
        self._rng = random.Random(seed)

    def next(self) -> SampleBatch:
        if self.n <= 1:
            return self.child.next()
        while len(self.buffer) < self.n:
            self.buffer.append(self.child.next())
        i = self._rng.randrange(len(self.buffer))
        out = self.buffer[i]
        self.buffer[i] = self.child.next()
        return out


class DatasetWriter(OutputWriter):
    """Buffers written batches and flushes them as a row-per-timestep Ray Data dataset
    (``output_config={"format": "json" | "parquet", "max_num_samples_per_file": n}``)."""

    def __init__(self, ioctx: Optional[IOContext] = None, compress_columns: Optional[List[str]] = None,
                 path: Optional[str] = None, fmt: Optional[str] = None, max_num_samples_per_file: int = 100000):
        cfg = (ioctx.config if ioctx is not None else {}) or {}
        out_cfg = cfg.get("output_config", {}) or {}
        self.path = path or cfg.get("output") or out_cfg.get("path")
        if not self.path:
            raise ValueError("DatasetWriter needs an output path")
        self.fmt = fmt or out_cfg.get("format", "json")
        self.max = int(out_cfg.get("max_num_samples_per_file", max_num_samples_per_file))
        self._pending: List[SampleBatch] = []
        self._n = 0
        self._files = 0

    def write(self, sample_batch: SampleBatch) -> None:
        self._pending.append(sample_batch)
        self._n += sample_batch.count
        if self._n >= self.max:
            self.flush()

    def flush(self) -> None:
        import os

        from .dataset_reader import write_dataset_rows

        if not self._pending:
            return
        write_dataset_rows(self._pending, os.path.join(self.path, f"part-{self._files:05d}"), self.fmt)
        self._files += 1
        self._pending, self._n = [], 0


class D4RLReader(InputReader):
    def __init__(self, *a, **k):
        raise ImportError("D4RLReader needs the `d4rl` package, which is not installed in this environment")


def get_offline_io_resource_bundles(config) -> List[Dict[str, float]]:
    """Resource bundles of the Ray Data read tasks behind ``input_="dataset"`` (one per parallel
    read, ``input_config["num_cpus_per_read_task"]`` CPUs each)."""
    cfg = config if isinstance(config, dict) else getattr(config, "to_dict", lambda: {})()
    if cfg.get("input") != "dataset" and cfg.get("input_") != "dataset":
        return []
    ic = cfg.get("input_config", {}) or {}
    par = int(ic.get("parallelism", cfg.get("num_env_runners", 0) or 1))
    return [{"CPU": float(ic.get("num_cpus_per_read_task", 0.5))} for _ in range(par)]


class FeatureImportance:
    """Permutation feature importance of a policy on logged data (reference
    offline/feature_importance.py): for each observation feature, the mean absolute change of
    the greedy action (or, for continuous actions, of the action vector) when that feature is
    shuffled across the batch, averaged over ``repeat`` shuffles."""

    def __init__(self, policy, repeat: int = 1, limit_fraction: float = 1.0, seed: Optional[int] = None):
        self.policy = policy
        self.repeat = int(repeat)
        self.limit_fraction = float(limit_fraction)
        self._rng = np.random.default_rng(seed)

    def _actions(self, obs):
        a, _, _ = self.policy.compute_actions(obs, explore=False)
        return np.asarray(a, dtype=np.float64).reshape(len(obs), -1)

    def estimate(self, batch: SampleBatch) -> Dict[str, float]:
        obs = np.asarray(batch[SampleBatch.OBS], dtype=np.float32)
        n = max(1, int(len(obs) * self.limit_fraction))
        obs = obs[:n]
        flat = obs.reshape(n, -1)
        base = self._actions(obs)
        out = {}
        for j in range(flat.shape[1]):
            deltas = []
            for _ in range(self.repeat):
                pert = flat.copy()
                pert[:, j] = pert[self._rng.permutation(n), j]
                deltas.append(np.abs(self._actions(pert.reshape(obs.shape)) - base).mean())
            out[f"feature_{j}"] = float(np.mean(deltas))
        return out

    def estimate_on_dataset(self, batch: SampleBatch, **kw) -> Dict[str, float]:
        return self.estimate(batch)
