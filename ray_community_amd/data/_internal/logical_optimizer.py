"""Logical-plan optimizer and physical planning of a Dataset's operator chain (reference:
``python/ray/data/_internal/logical/rules/limit_pushdown.py:13`` ``LimitPushdownRule`` and
``operator_fusion.py:34`` ``OperatorFusionRule``).

A Dataset's plan is a linear chain of op dicts (``dataset.py``). Two rule families:

* **Limit pushdown**: a ``limit`` moves upstream past every operator that maps one row to one
  row (``map``, column projections / additions / renames) and consecutive limits fuse into
  ``limit(min)``. ``ds.map(f).limit(10)`` then runs ``f`` only on the first rows instead of on
  every block the read produced before the limit stopped upstream work.
* **Operator fusion** (physical planning): consecutive task-compute maps with compatible resource
  requests run as ONE task per block (one block round trip through the object store instead of
  one per operator); a task-compute chain directly upstream of an actor-pool map runs inside
  the pool's actors when both need nothing but CPU. Incompatible neighbours (different GPU or
  custom-resource requests, scheduling strategies or runtime envs) stay separate operators: in
  particular a CPU chain is NOT absorbed into a GPU actor pool, whose few actors are sized for
  the GPU stage (measured: CPU image synthesis absorbed into the 2-actor GPU pool of
  ``bench_data_serve.py`` ran the pipeline at 25.6k instead of 35k images/s).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

# ops that emit exactly one output row per input row (reference: can_modify_num_rows = False)
ROW_PRESERVING = {"map", "add_column", "drop_columns", "select_columns", "rename_columns"}
MAP_KINDS = {"map_batches", "map", "flat_map", "filter", "add_column", "drop_columns", "select_columns",
             "rename_columns"}
_PLACEMENT_KEYS = ("resources", "memory", "scheduling_strategy", "runtime_env", "accelerator_type")


def push_down_limits(ops: List[Dict], enabled: bool = True) -> Tuple[List[Dict], List[str]]:
    """(rewritten chain, rules that changed it)."""
    ops = [dict(o) for o in ops]
    if not enabled:
        return ops, []
    applied = []
    changed = True
    while changed:
        changed = False
        for i in range(1, len(ops)):
            if ops[i]["kind"] != "limit":
                continue
            prev = ops[i - 1]
            if prev["kind"] == "limit":
                ops[i - 1] = {"kind": "limit", "n": min(int(prev["n"]), int(ops[i]["n"]))}
                del ops[i]
                applied.append("LimitFusion")
                changed = True
                break
            if prev["kind"] in ROW_PRESERVING:
                ops[i - 1], ops[i] = ops[i], prev
                applied.append("LimitPushdown")
                changed = True
                break
    return ops, sorted(set(applied), key=applied.index)


def _placement(op: Dict) -> Tuple:
    rr = op.get("ray_remote_args") or {}
    return (float(op.get("num_gpus") or 0),) + tuple(repr(rr.get(k)) for k in _PLACEMENT_KEYS)


def compatible(a: Dict, b: Dict) -> bool:
    """Two task-compute maps can share a task: same GPU share and placement-relevant remote args
    (CPU requests may differ: the fused task takes the larger)."""
    return _placement(a) == _placement(b)


def _cpu_only(chain: List[Dict]) -> bool:
    return all(_placement(o) == _placement({}) for o in chain)


def plan_stages(ops: List[Dict], fuse: bool = True) -> List[Tuple]:
    """Physical stages: ("task", chain) | ("actor", op, pre_chain) | ("limit", n) | ("alltoall", op)
    | ("nary", op) (streaming union / zip with other datasets).
    ``fuse=False``: one stage per operator."""
    stages: List[Tuple] = []
    chain: List[Dict] = []

    def flush():
        nonlocal chain
        if chain:
            stages.append(("task", chain))
            chain = []

    for op in ops:
        k = op["kind"]
        if k in MAP_KINDS and op.get("compute") != "actors":
            if chain and (not fuse or not compatible(chain[-1], op)):
                flush()
            chain.append(op)
            continue
        if k in MAP_KINDS:  # actor pool: absorb an upstream CPU-only task chain (CPU-only pool)
            pre = []
            if fuse and chain and _cpu_only(chain) and _cpu_only([op]):
                pre, chain = chain, []
            flush()
            stages.append(("actor", op, pre))
            continue
        flush()
        if k == "limit":
            stages.append(("limit", int(op["n"])))
        elif k == "alltoall":
            stages.append(("alltoall", op))
        elif k in ("union", "zip"):
            stages.append(("nary", op))
        else:
            raise ValueError(f"unknown operator kind {k!r}")
    flush()
    return stages


def describe(stages: List[Tuple], name_of) -> str:
    parts = ["Input"]
    for st in stages:
        if st[0] == "task":
            parts.append("TaskMap[" + "->".join(name_of(o) for o in st[1]) + "]")
        elif st[0] == "actor":
            pre = "->".join(name_of(o) for o in st[2])
            parts.append("ActorPoolMap[" + (pre + "->" if pre else "") + name_of(st[1]) + "]")
        elif st[0] == "limit":
            parts.append(f"Limit[{st[1]}]")
        else:
            parts.append(st[1].get("name", "AllToAll"))
    return " -> ".join(parts)
