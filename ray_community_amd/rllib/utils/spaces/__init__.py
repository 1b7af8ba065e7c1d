"""Minimal gym-compatible spaces (gymnasium is not installed in this environment)."""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


class Space:
    shape = ()
    dtype = None

    def sample(self):
        raise NotImplementedError

    def contains(self, x) -> bool:
        raise NotImplementedError


class Discrete(Space):
    def __init__(self, n: int, seed: Optional[int] = None):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return int(self._rng.integers(self.n))

    def contains(self, x):
        try:
            return 0 <= int(x) < self.n
        except (TypeError, ValueError):
            return False

    def __repr__(self):
        return f"Discrete({self.n})"

    def __eq__(self, o):
        return isinstance(o, Discrete) and o.n == self.n


class Box(Space):
    def __init__(self, low, high, shape: Optional[Sequence[int]] = None, dtype=np.float32, seed=None):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), self.shape).copy()
        self._rng = np.random.default_rng(seed)

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self._rng.integers(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return self._rng.uniform(lo, hi, size=self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Tuple(Space):
    """A tuple of spaces (grouped agents' observations / actions)."""

    def __init__(self, spaces: Sequence[Space]):
        self.spaces = tuple(spaces)
        self.shape = None
        self.dtype = None

    def sample(self):
        return tuple(s.sample() for s in self.spaces)

    def contains(self, x) -> bool:
        return isinstance(x, (tuple, list)) and len(x) == len(self.spaces) and all(
            s.contains(v) for s, v in zip(self.spaces, x))

    def __len__(self):
        return len(self.spaces)

    def __getitem__(self, i):
        return self.spaces[i]

    def __repr__(self):
        return "Tuple(" + ", ".join(repr(s) for s in self.spaces) + ")"

    def __eq__(self, o):
        return isinstance(o, Tuple) and o.spaces == self.spaces


class Dict(Space):
    """A dict of named spaces."""

    def __init__(self, spaces=None, **kw):
        self.spaces = dict(spaces or {}, **kw)
        self.shape = None
        self.dtype = None

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def contains(self, x) -> bool:
        return isinstance(x, dict) and set(x) == set(self.spaces) and all(
            self.spaces[k].contains(v) for k, v in x.items())

    def __getitem__(self, k):
        return self.spaces[k]

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k}: {s!r}" for k, s in self.spaces.items()) + ")"
