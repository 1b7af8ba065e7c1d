"""Training/tuning result (reference: ``python/ray/air/result.py``)."""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple


@dataclass
class Result:
    metrics: Optional[Dict[str, Any]]
    checkpoint: Optional[Any]
    error: Optional[BaseException] = None
    path: Optional[str] = None
    metrics_history: List[Dict[str, Any]] = field(default_factory=list)
    best_checkpoints: List[Tuple[Any, Dict[str, Any]]] = field(default_factory=list)
    filesystem: Any = None

    @property
    def config(self):
        return (self.metrics or {}).get("config")

    @property
    def metrics_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.metrics_history) if self.metrics_history else None

    def get_best_checkpoint(self, metric: str, mode: str):
        """The kept checkpoint whose reported ``metric`` is best (``mode`` "max" / "min"); None if
        no kept checkpoint reported it."""
        if mode not in ("max", "min"):
            raise ValueError("mode must be 'max' or 'min'")
        scored = [(m[metric], c) for c, m in self.best_checkpoints if isinstance(m, dict) and metric in m]
        if not scored:
            return None
        pick = max if mode == "max" else min
        return pick(scored, key=lambda t: t[0])[1]

    @classmethod
    def from_path(cls, path: str) -> "Result":
        from ..train._checkpoint import Checkpoint

        hist = []
        p = os.path.join(path, "result.json")
        if os.path.exists(p):
            with open(p) as f:
                hist = [json.loads(l) for l in f if l.strip()]
        ckpts = sorted(d for d in os.listdir(path) if d.startswith("checkpoint_")) if os.path.isdir(path) else []
        ck = Checkpoint.from_directory(os.path.join(path, ckpts[-1])) if ckpts else None
        return cls(metrics=hist[-1] if hist else None, checkpoint=ck, path=path, metrics_history=hist)

    def __repr__(self):
        return f"Result(metrics={self.metrics}, path={self.path}, checkpoint={self.checkpoint}, error={self.error!r})"
