"""Task bodies of Dataset execution (reference: ``data/_internal/execution/operators/
{map_operator,actor_pool_map_operator}.py``, ``planner/exchange``); the scheduling loop that runs
them is ``streaming_executor.py``.

* consecutive task-compute map operators are FUSED into one remote task per block (``_run_chain``);
* actor-pool operators (callable-class UDFs, ``concurrency=``, ``num_gpus=``) run ``_MapActor``
  (GPU preprocessing runs here);
* all-to-all operators (repartition, shuffle, sort, groupby) are two-phase map/reduce exchanges.
Each task returns ``(block, metadata)`` as two objects so counts/limits need no block fetches.
"""
from __future__ import annotations

import collections
import itertools
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

import numpy as np

from ..block import BlockAccessor, concat_blocks, normalize_block
from ..exceptions import call_user_fn


def _meta(block) -> Dict:
    a = BlockAccessor(block)
    return {"num_rows": a.num_rows(), "size_bytes": a.size_bytes()}


# ------------------------------------------------------------------------------ map functions
def _apply_map_op(block, op) -> List:
    """Apply one map operator to a block; returns a list of output blocks."""
    kind = op["kind"]
    fn = op.get("fn")
    acc = BlockAccessor(block)
    if kind == "map_batches":
        fmt = op.get("batch_format", "default")
        bs = op.get("batch_size")
        n = acc.num_rows()
        outs = []
        if n == 0:
            return []
        step = n if bs in (None, "default") or bs <= 0 else bs
        for s in range(0, n, step):
            batch = BlockAccessor(acc.slice(s, min(n, s + step))).to_batch(fmt)
            res = call_user_fn(fn, batch, *op.get("fn_args", ()), **op.get("fn_kwargs", {}))
            if hasattr(res, "__next__") and not isinstance(res, dict):
                outs.extend(normalize_block(r) for r in res)
            else:
                outs.append(normalize_block(res))
        return outs
    if kind == "map":
        rows = [call_user_fn(fn, r, *op.get("fn_args", ()), **op.get("fn_kwargs", {})) for r in acc.iter_rows()]
        from ..block import rows_to_block

        return [rows_to_block(rows)]
    if kind == "flat_map":
        rows = []
        for r in acc.iter_rows():
            rows.extend(call_user_fn(fn, r, *op.get("fn_args", ()), **op.get("fn_kwargs", {})))
        from ..block import rows_to_block

        return [rows_to_block(rows)]
    if kind == "filter":
        if op.get("expr") is not None:
            import pandas as pd  # noqa

            df = acc.to_pandas()
            return [normalize_block(df.query(op["expr"]))]
        mask = np.array([bool(call_user_fn(fn, r)) for r in acc.iter_rows()], dtype=bool)
        return [acc.take(np.nonzero(mask)[0])]
    if kind == "add_column":
        b = acc.to_pandas() if op.get("batch_format", "pandas") == "pandas" else acc.to_numpy()
        col = call_user_fn(fn, b)
        if hasattr(b, "assign"):
            b = b.assign(**{op["col"]: col})
        else:
            b = dict(b)
            b[op["col"]] = np.asarray(col)
        return [normalize_block(b)]
    if kind == "drop_columns":
        d = acc.to_numpy() if not hasattr(block, "drop") else None
        if d is None:
            return [block.drop(op["cols"])]
        return [{k: v for k, v in d.items() if k not in op["cols"]}]
    if kind == "select_columns":
        if hasattr(block, "select"):
            return [block.select(op["cols"])]
        d = acc.to_numpy()
        return [{k: d[k] for k in op["cols"]}]
    if kind == "rename_columns":
        d = acc.to_numpy()
        return [{op["mapping"].get(k, k): v for k, v in d.items()}]
    raise ValueError(f"unknown map op {kind}")


def _run_chain(block, ops) -> Tuple[Any, Dict]:
    blocks = [block]
    for op in ops:
        nb = []
        for b in blocks:
            nb.extend(_apply_map_op(b, op))
        blocks = nb
    out = concat_blocks(blocks) if len(blocks) != 1 else blocks[0]
    return out, _meta(out)


def _read_task(read_fn) -> Tuple[Any, Dict]:
    b = normalize_block(read_fn())
    return b, _meta(b)


class _MapActor:
    def __init__(self, cls, ctor_args, ctor_kwargs, ops_before, ops_after, op):
        self.udf = cls(*ctor_args, **ctor_kwargs)
        self.ops_before = ops_before
        self.ops_after = ops_after
        self.op = dict(op)
        self.op["fn"] = self.udf

    def process(self, block):
        blocks = [block]
        for o in self.ops_before + [self.op] + self.ops_after:
            nb = []
            for b in blocks:
                nb.extend(_apply_map_op(b, o))
            blocks = nb
        out = concat_blocks(blocks) if len(blocks) != 1 else blocks[0]
        return out, _meta(out)

    def ready(self):
        return True


# ------------------------------------------------------------------------------ stages
def _remote_fn(f, opts):
    from ...remote_function import RemoteFunction

    return RemoteFunction(f, {"num_returns": 2, **opts})


def _truncate(block, k):
    out = BlockAccessor(block).slice(0, k)
    return out, _meta(out)


def _zip_columns(a, b):
    da = BlockAccessor(a).to_numpy()
    db = BlockAccessor(b).to_numpy()
    out = dict(da)
    for k, v in db.items():
        out[k if k not in out else f"{k}_1"] = v
    return out


def _zip_slices(a, a0, b, b0, n):
    """Rows [a0, a0+n) of ``a`` side by side with rows [b0, b0+n) of ``b`` (streaming zip)."""
    out = _zip_columns(BlockAccessor(a).slice(a0, a0 + n), BlockAccessor(b).slice(b0, b0 + n))
    return out, _meta(out)


# ------------------------------------------------------------------------------ exchanges
def _split_by_ranges(block, start_row, bounds):
    """Slice ``block`` (global rows [start_row, start_row+n)) into len(bounds)-1 pieces."""
    acc = BlockAccessor(block)
    n = acc.num_rows()
    out = []
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        s = max(lo - start_row, 0)
        e = min(hi - start_row, n)
        out.append(acc.slice(s, e) if e > s else acc.slice(0, 0))
    return out


def _split_random(block, k, seed):
    acc = BlockAccessor(block)
    n = acc.num_rows()
    rng = np.random.default_rng(seed)
    assign = rng.integers(0, k, n)
    return [acc.take(np.nonzero(assign == j)[0]) for j in range(k)]


def _split_by_key_bounds(block, key, bounds, descending):
    acc = BlockAccessor(block)
    d = acc.to_numpy()
    if key not in d:  # empty block (e.g. an empty groupby partition)
        return [acc.slice(0, 0) for _ in range(len(bounds) + 1)]
    keys = d[key]
    order = np.argsort(keys, kind="stable")
    if descending:
        order = order[::-1]
    part = np.searchsorted(bounds, keys, side="right") if len(bounds) else np.zeros(len(keys), dtype=np.int64)
    if descending:
        part = len(bounds) - part
    out = []
    for j in range(len(bounds) + 1):
        idx = np.nonzero(part == j)[0]
        out.append(acc.take(idx))
    return out


def _split_by_hash(block, keys, k):
    acc = BlockAccessor(block)
    if acc.num_rows() == 0:
        return [acc.slice(0, 0) for _ in range(k)]
    df = acc.to_pandas()
    import pandas as pd

    h = pd.util.hash_pandas_object(df[keys], index=False).to_numpy() % k
    return [acc.take(np.nonzero(h == j)[0]) for j in range(k)]


def _reduce_concat(*pieces, shuffle_seed=None, sort_key=None, descending=False):
    b = concat_blocks(list(pieces))
    acc = BlockAccessor(b)
    if shuffle_seed is not None and acc.num_rows() > 0:
        perm = np.random.default_rng(shuffle_seed).permutation(acc.num_rows())
        b = acc.take(perm)
    if isinstance(sort_key, list) and acc.num_rows() > 0:  # several keys: lexicographic, per-key order
        df = BlockAccessor(b).to_pandas().reset_index(drop=True)
        order = df.sort_values(sort_key, ascending=[not d for d in descending], kind="mergesort").index.to_numpy()
        b = BlockAccessor(b).take(order)
    elif sort_key is not None and acc.num_rows() > 0:
        d = BlockAccessor(b).to_numpy()
        order = np.argsort(d[sort_key], kind="stable")
        if descending:
            order = order[::-1]
        b = BlockAccessor(b).take(order)
    return b, _meta(b)


def _reduce_groupby(*pieces, keys=None, aggs=None, map_groups=None, batch_format="pandas"):
    b = concat_blocks(list(pieces))
    acc = BlockAccessor(b)
    if acc.num_rows() == 0:
        return {}, {"num_rows": 0, "size_bytes": 0}
    df = acc.to_pandas()
    if map_groups is not None:
        outs = []
        gb = df.groupby(keys, sort=True) if keys else [(None, df)]
        for _, g in gb:
            batch = normalize_block(g.reset_index(drop=True))
            res = map_groups(BlockAccessor(batch).to_batch(batch_format))
            outs.append(normalize_block(res))
        out = concat_blocks(outs)
        return out, _meta(out)
    import pandas as pd

    if keys:
        gb = df.groupby(keys, sort=True)
        res = {}
        for agg in aggs:
            res[agg.name] = agg.pandas_agg(gb)
        out_df = pd.DataFrame(res).reset_index()
    else:
        out_df = pd.DataFrame({agg.name: [agg.pandas_agg_all(df)] for agg in aggs})
    out = normalize_block(out_df)
    return out, _meta(out)


def exchange(refs_metas: List[Tuple[Any, Any]], num_out: int, map_fn, map_args_per_block, reduce_fn,
             reduce_kwargs_per_out) -> List[Tuple[Any, Any]]:
    """Generic two-phase exchange: each input block -> num_out pieces; reducer j concats pieces j."""
    from ...remote_function import RemoteFunction

    if num_out <= 0:
        return []
    if num_out == 1:
        base = map_fn

        def map_fn(*a):  # a single return is the value itself, not a 1-list
            return base(*a)[0]

    mfn = RemoteFunction(map_fn, {"num_returns": num_out, "num_cpus": 1})
    pieces = []
    for (b, _), args in zip(refs_metas, map_args_per_block):
        r = mfn.remote(b, *args)
        pieces.append(r if isinstance(r, list) else [r])
    rfn = RemoteFunction(reduce_fn, {"num_returns": 2, "num_cpus": 1})
    out = []
    for j in range(num_out):
        col = [p[j] for p in pieces]
        out.append(tuple(rfn.remote(*col, **reduce_kwargs_per_out[j])))
    return out
