"""Progress bars from tasks and actors (reference: python/ray/experimental/tqdm_ray.py).

``tqdm`` here has the tqdm call surface (``update``, ``set_description``, ``close``, iteration)
and writes throttled one-line progress records (``desc: n/total``) to stdout; worker stdout is
forwarded to the driver by the log monitor, so the driver sees every remote bar's progress
prefixed with the producing actor / task, without a shared terminal."""
from __future__ import annotations

import sys
import time
from typing import Iterable, Optional


class tqdm:  # noqa: N801 (reference name)
    def __init__(self, iterable: Optional[Iterable] = None, desc: Optional[str] = None,
                 total: Optional[int] = None, unit: str = "it", position: Optional[int] = None,
                 flush_interval_s: float = 1.0, **kwargs):
        self.iterable = iterable
        self.desc = desc or ""
        self.total = total if total is not None else (len(iterable) if hasattr(iterable, "__len__") else None)
        self.unit = unit
        self.n = 0
        self._interval = float(flush_interval_s)
        self._last = 0.0
        self._t0 = time.time()
        self._closed = False

    def _emit(self, force: bool = False) -> None:
        now = time.time()
        if not force and now - self._last < self._interval:
            return
        self._last = now
        rate = self.n / max(now - self._t0, 1e-9)
        tot = f"/{self.total}" if self.total is not None else ""
        sys.stdout.write(f"{self.desc}: {self.n}{tot} {self.unit} [{rate:.1f} {self.unit}/s]\n")
        sys.stdout.flush()

    def update(self, n: int = 1) -> None:
        self.n += n
        self._emit()

    def set_description(self, desc: Optional[str] = None, refresh: bool = True) -> None:
        self.desc = desc or ""

    def refresh(self) -> None:
        self._emit(force=True)

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            self._emit(force=True)

    def __iter__(self):
        for x in self.iterable:
            yield x
            self.update(1)
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def safe_print(*args, **kwargs) -> None:
    print(*args, **kwargs)


__all__ = ["tqdm", "safe_print"]
