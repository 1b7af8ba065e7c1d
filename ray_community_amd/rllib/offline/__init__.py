"""Offline data I/O (reference: ``rllib/offline/json_writer.py``, ``json_reader.py``,
``dataset_reader.py``, ``estimators/``).

Batches are written as JSON lines (one flattened SampleBatch per line, arrays as nested lists);
the reader samples whole lines or concatenates them into train batches.
"""
from __future__ import annotations

import glob
import json
import os
import random
import time
from typing import List, Optional

import numpy as np

from ..policy.sample_batch import SampleBatch, concat_samples


class JsonWriter:
    def __init__(self, path: str, max_file_size: int = 64 * 1024 * 1024):
        os.makedirs(path, exist_ok=True)
        self.path = path
        self.max = max_file_size
        self._f = None
        self._idx = 0

    def _file(self):
        if self._f is None or self._f.tell() > self.max:
            if self._f is not None:
                self._f.close()
            name = os.path.join(self.path, f"output-{time.strftime('%Y-%m-%d_%H-%M-%S')}_worker-{os.getpid()}_"
                                           f"{self._idx}.json")
            self._idx += 1
            self._f = open(name, "w")
        return self._f

    def write(self, batch: SampleBatch):
        b = batch.flatten() if getattr(batch, "fragment_shape", None) is not None else batch
        row = {k: (np.asarray(v).tolist()) for k, v in b.items()}
        if getattr(batch, "fragment_shape", None) is not None:
            row["_fragment_shape"] = list(batch.fragment_shape)
        f = self._file()
        f.write(json.dumps(row) + "\n")
        f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


class JsonReader:
    def __init__(self, inputs, seed: Optional[int] = None):
        if isinstance(inputs, str):
            inputs = sorted(glob.glob(os.path.join(inputs, "*.json"))) if os.path.isdir(inputs) else \
                sorted(glob.glob(inputs))
        self.files = list(inputs)
        if not self.files:
            raise ValueError(f"no offline input files found in {inputs}")
        self.batches: List[SampleBatch] = []
        for fn in self.files:
            with open(fn) as f:
                for line in f:
                    if line.strip():
                        self.batches.append(self._parse(json.loads(line)))
        self._rng = random.Random(seed)

    @staticmethod
    def _parse(row) -> SampleBatch:
        fs = row.pop("_fragment_shape", None)
        b = SampleBatch({k: np.asarray(v) for k, v in row.items()})
        if fs is not None:
            N, T = fs
            # restore env-major [N, T] blocks so episode boundaries stay contiguous per env
            b = SampleBatch({k: v.reshape((N, T) + v.shape[1:]) for k, v in b.items()})
            b.fragment_shape = (N, T)
        return b

    def next(self) -> SampleBatch:
        return self._rng.choice(self.batches)

    def sample(self, n_min: int) -> SampleBatch:
        out, c = [], 0
        while c < n_min:
            b = self.next()
            out.append(b)
            c += b.count
        return concat_samples(out)

    def __iter__(self):
        return iter(self.batches)


from .dataset_reader import DatasetReader, get_dataset_and_shards, write_dataset_rows  # noqa: E402
from .io import (D4RLReader, DatasetWriter, FeatureImportance, InputReader, IOContext, MixedInput,  # noqa: E402
                 NoopOutput, OutputWriter, ShuffledInput, get_offline_io_resource_bundles)
