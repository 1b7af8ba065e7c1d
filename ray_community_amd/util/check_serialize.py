"""Find what makes an object unserializable (reference: ``python/ray/util/check_serialize.py``).

Walks closures, globals referenced by functions, and object attributes depth-first, reporting the
innermost members that fail to pickle with the framework's serializer."""
from __future__ import annotations

import inspect
from typing import Any, Optional, Set, Tuple


class FailureTuple:
    def __init__(self, obj, name, parent):
        self.obj = obj
        self.name = name
        self.parent = parent

    def __repr__(self):
        return f"FailTuple({self.name} [obj={self.obj}, parent={self.parent}])"

    def __eq__(self, other):
        return isinstance(other, FailureTuple) and self.name == other.name

    def __hash__(self):
        return hash(self.name)


def _serializable(obj) -> bool:
    from .._private import serialization as ser

    try:
        ser.serialize(obj)
        return True
    except Exception:
        return False


def _children(obj):
    if inspect.isfunction(obj):
        cv = inspect.getclosurevars(obj)
        yield from cv.nonlocals.items()
        yield from cv.globals.items()
        return
    if inspect.ismethod(obj):
        yield "__self__", obj.__self__
        yield "__func__", obj.__func__
        return
    d = getattr(obj, "__dict__", None)
    if isinstance(d, dict):
        yield from d.items()


def inspect_serializability(base_obj: Any, name: Optional[str] = None, depth: int = 3,
                            print_file=None) -> Tuple[bool, Set[FailureTuple]]:
    """Returns ``(serializable, failures)``; ``failures`` holds the innermost offending members."""
    name = name or getattr(base_obj, "__name__", repr(base_obj)[:60])
    failures: Set[FailureTuple] = set()

    def walk(obj, nm, parent, d):
        if _serializable(obj):
            return True
        found = False
        if d > 0:
            for cname, child in _children(obj):
                if not walk(child, cname, obj, d - 1):
                    found = True
        if not found:
            failures.add(FailureTuple(obj, nm, parent))
        return False

    ok = walk(base_obj, name, None, depth)
    if print_file is not None and not ok:
        for f in failures:
            print(f"  {f.name}: {type(f.obj).__name__} is not serializable", file=print_file)
    return ok, failures
