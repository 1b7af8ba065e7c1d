"""Search-space primitives (reference: ``python/ray/tune/search/sample.py``)."""
from __future__ import annotations

import math
import random
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np


class Domain:
    def sample(self, spec=None, size=1, random_state=None):
        rng = random_state if random_state is not None else np.random
        out = [self._sample_one(rng, spec) for _ in range(size)]
        return out[0] if size == 1 else out

    def _sample_one(self, rng, spec):
        raise NotImplementedError

    def is_grid(self):
        return False

    def is_function(self):
        return False

    @property
    def domain_str(self):
        return repr(self)


class Categorical(Domain):
    def __init__(self, categories: Sequence):
        self.categories = list(categories)

    def _sample_one(self, rng, spec):
        i = rng.randint(len(self.categories)) if hasattr(rng, "randint") else random.randrange(len(self.categories))
        v = self.categories[int(i)]
        return v.sample(spec) if isinstance(v, Domain) else v

    def __repr__(self):
        return f"choice({self.categories})"


class Float(Domain):
    def __init__(self, lower, upper, log=False, q=None, base=10, normal=False, mean=0.0, sd=1.0):
        self.lower, self.upper, self.log, self.q, self.base = lower, upper, log, q, base
        self.normal, self.mean, self.sd = normal, mean, sd
        if not normal:
            if lower >= upper and not (q and lower == upper):
                raise ValueError("lower must be < upper")
            if log and lower <= 0:
                raise ValueError("loguniform lower bound must be > 0")

    def _sample_one(self, rng, spec):
        if self.normal:
            v = rng.normal(self.mean, self.sd)
        elif self.log:
            lb = math.log(self.lower) / math.log(self.base)
            ub = math.log(self.upper) / math.log(self.base)
            v = self.base ** rng.uniform(lb, ub)
        else:
            v = rng.uniform(self.lower, self.upper)
        if self.q:
            v = float(np.round(v / self.q) * self.q)
            if not self.normal:
                v = min(max(v, self.lower), self.upper)
        return float(v)

    def __repr__(self):
        return f"{'loguniform' if self.log else 'uniform'}({self.lower}, {self.upper})"


class Integer(Domain):
    def __init__(self, lower, upper, log=False, q=None, base=10):
        self.lower, self.upper, self.log, self.q, self.base = lower, upper, log, q, base
        if lower >= upper:
            raise ValueError("lower must be < upper")

    def _sample_one(self, rng, spec):
        if self.log:
            lb = math.log(self.lower) / math.log(self.base)
            ub = math.log(self.upper) / math.log(self.base)
            v = int(self.base ** rng.uniform(lb, ub))
        else:
            v = int(rng.randint(self.lower, self.upper))
        if self.q:  # quantised variants include the upper bound (reference semantics)
            return min(max(int(round(v / self.q) * self.q), self.lower), self.upper)
        return min(max(v, self.lower), self.upper - 1)

    def __repr__(self):
        return f"randint({self.lower}, {self.upper})"


class Function(Domain):
    def __init__(self, func: Callable):
        self.func = func

    def is_function(self):
        return True

    def _sample_one(self, rng, spec):
        import inspect

        try:
            n = len(inspect.signature(self.func).parameters)
        except (TypeError, ValueError):
            n = 1
        return self.func(spec) if n >= 1 else self.func()


def choice(categories):
    return Categorical(categories)


def uniform(lower, upper):
    return Float(lower, upper)


def quniform(lower, upper, q):
    return Float(lower, upper, q=q)


def loguniform(lower, upper, base=10):
    return Float(lower, upper, log=True, base=base)


def qloguniform(lower, upper, q, base=10):
    return Float(lower, upper, log=True, q=q, base=base)


def randn(mean=0.0, sd=1.0):
    return Float(None, None, normal=True, mean=mean, sd=sd)


def qrandn(mean, sd, q):
    return Float(None, None, normal=True, mean=mean, sd=sd, q=q)


def randint(lower, upper):
    return Integer(lower, upper)


def qrandint(lower, upper, q=1):
    return Integer(lower, upper, q=q)


def lograndint(lower, upper, base=10):
    return Integer(lower, upper, log=True, base=base)


def qlograndint(lower, upper, q, base=10):
    return Integer(lower, upper, log=True, q=q, base=base)


def sample_from(func):
    return Function(func)


def grid_search(values):
    return {"grid_search": list(values)}
