"""Offline input through Ray Data (reference: ``rllib/offline/dataset_reader.py:179``
``DatasetReader`` and ``get_dataset_and_shards``).

The dataset's rows are timesteps (columns ``obs``, ``actions``, ``rewards``, ``terminateds``,
optionally ``truncateds``, ``eps_id``, ``action_logp`` / ``action_prob``, ``new_obs``). The reader
streams it with ``iter_batches`` (re-iterating, i.e. re-executing, once exhausted, so a shuffled
dataset gives a new order every pass) and hands out ``SampleBatch``es of ``batch_size`` rows; when
the rows carry rewards and episode boundaries, the batch also gets ``returns`` (discounted
reward-to-go inside the batch) for MARWIL's advantage weights.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..policy.sample_batch import SampleBatch, concat_samples


def _read(fmt: str, paths, **kw):
    from ... import data

    fn = {"json": data.read_json, "parquet": data.read_parquet, "csv": data.read_csv,
          "numpy": data.read_numpy}.get(fmt)
    if fn is None:
        raise ValueError(f"unsupported offline dataset format {fmt!r}")
    return fn(paths, **kw)


def get_dataset_and_shards(config, num_workers: int = 0) -> Tuple[Any, List[Any]]:
    """The offline Dataset of ``config.input_config`` (``{"dataset": ds}`` or
    ``{"format": ..., "paths": ...}``) and ``num_workers`` shards of it (or [ds])."""
    ic = dict(getattr(config, "input_config", None) or {})
    ds = ic.get("dataset")
    if ds is None:
        if "paths" not in ic:
            raise ValueError('input_="dataset" needs input_config={"format": ..., "paths": ...} or {"dataset": ds}')
        ds = _read(ic.get("format", "json"), ic["paths"])
    if num_workers > 1:
        return ds, ds.split(num_workers, equal=True)
    return ds, [ds]


class DatasetReader:
    def __init__(self, ds, batch_size: int = 1000, gamma: float = 0.99, shuffle_buffer: Optional[int] = None,
                 seed: Optional[int] = None):
        self.ds = ds
        self.batch_size = int(batch_size)
        self.gamma = float(gamma)
        self.shuffle_buffer = shuffle_buffer
        self.seed = seed
        self._it = None
        self.epochs = 0

    def _batches(self):
        while True:
            self.epochs += 1
            n = 0
            for b in self.ds.iter_batches(batch_size=self.batch_size, batch_format="numpy",
                                          local_shuffle_buffer_size=self.shuffle_buffer,
                                          local_shuffle_seed=self.seed):
                n += 1
                yield b
            if n == 0:
                raise ValueError("the offline dataset is empty")

    def next(self) -> SampleBatch:
        if self._it is None:
            self._it = self._batches()
        cols = next(self._it)
        b = SampleBatch({k: np.stack(v) if v.dtype == object else np.asarray(v) for k, v in cols.items()})
        if SampleBatch.REWARDS in b and "returns" not in b:
            b["returns"] = self._returns(b)
        return b

    def _returns(self, b: SampleBatch) -> np.ndarray:
        r = np.asarray(b[SampleBatch.REWARDS], np.float64)
        done = np.asarray(b.get(SampleBatch.TERMINATEDS, np.zeros(len(r), bool)), bool)
        if SampleBatch.TRUNCATEDS in b:
            done = done | np.asarray(b[SampleBatch.TRUNCATEDS], bool)
        if SampleBatch.EPS_ID in b:
            e = np.asarray(b[SampleBatch.EPS_ID])
            done = done | np.concatenate([e[1:] != e[:-1], [True]])
        out = np.empty_like(r)
        acc = 0.0
        for t in range(len(r) - 1, -1, -1):
            acc = r[t] + (0.0 if done[t] else self.gamma * acc)
            out[t] = acc
        return out.astype(np.float32)

    def sample(self, n_min: int) -> SampleBatch:
        out, c = [], 0
        while c < n_min:
            b = self.next()
            out.append(b)
            c += b.count
        return concat_samples(out) if len(out) > 1 else out[0]

    def __iter__(self):
        while True:
            yield self.next()


def write_dataset_rows(batches, path: str, fmt: str = "parquet"):
    """Logged SampleBatches (env-major fragments or flat) -> a row-per-timestep dataset on disk
    with ``eps_id`` per row (episode ids are (fragment env row, episode count) pairs)."""
    from ... import data
    from .estimators.off_policy_estimator import split_by_episode

    rows: Dict[str, list] = {}
    eid = 0
    for b in batches:
        for ep in split_by_episode(b):
            n = len(ep[SampleBatch.REWARDS])
            for k, v in ep.items():
                rows.setdefault(k, []).extend(list(np.asarray(v)))
            rows.setdefault(SampleBatch.EPS_ID, []).extend([eid] * n)
            eid += 1
    ds = data.from_items([{k: rows[k][i] for k in rows} for i in range(len(rows[SampleBatch.REWARDS]))])
    getattr(ds, f"write_{fmt}")(path)
    return path
