"""A simple map/reduce shuffle over tasks and the object store (reference:
``python/ray/experimental/shuffle.py`` -- ``simple_shuffle`` and its ``python -m`` driver, used by the
reference's object-store scalability tests).

``simple_shuffle`` redistributes M input partitions into N output partitions with one wave of map
tasks (map i reads input partition i and routes every item to an output partition) followed by one
wave of reduce tasks (reduce j consumes what every map routed to j): O(M * N) objects in flight.
Large items go through the shared-memory store (and are spilled when it fills), small ones stay
inline in the owner. Map outputs are written by an ``ObjectStoreWriter``: the default puts each
item as its own object and passes the refs (the reduce side streams them one by one with
``wait``); ``ObjectStoreWriterNonStreaming`` passes the items themselves.

    python -m ray_community_amd.experimental.shuffle --num-partitions 8 --partition-size 50e6
"""
from __future__ import annotations

import argparse
import json
import time
from typing import Any, Callable, Iterable, List, Optional

import numpy as np

from .._private import worker as _w

PartitionID = int


class ObjectStoreWriter:
    """Collects one map task's items for one output partition. ``add`` puts each item into the
    object store right away (a streaming reducer can fetch it as soon as the map finishes);
    subclass it to batch small records into larger objects."""

    def __init__(self):
        self.results: List[Any] = []

    def add(self, item: Any) -> None:
        self.results.append(_w.put(item))

    def finish(self) -> List[Any]:
        return self.results


class ObjectStoreWriterNonStreaming(ObjectStoreWriter):
    """Keeps the items themselves: they travel as the map task's return value."""

    def add(self, item: Any) -> None:
        self.results.append(item)


def round_robin_partitioner(input_stream: Iterable[Any], num_partitions: int):
    """Item k of the stream goes to output partition k mod ``num_partitions``."""
    for k, item in enumerate(input_stream):
        yield k % num_partitions, item


def _map(reader, partitioner, writer_cls, n_out, i):
    writers = [writer_cls() for _ in range(n_out)]
    for j, item in partitioner(reader(i), n_out):
        writers[j].add(item)
    outs = [w.finish() for w in writers]
    return outs if n_out > 1 else outs[0]


def _reduce(writer, streaming, j, *map_outputs):
    # map_outputs[i]: what map i routed here (refs when streaming, the items otherwise)
    flat = [x for part in map_outputs for x in part]
    return writer(j, flat)


class ShuffleProgress:
    """Map / reduce completion counts of a running shuffle (the reference's ``_StatusTracker``,
    here polled from the driver with non-blocking waits instead of a tracker actor)."""

    def __init__(self, map_refs, reduce_refs):
        self._map, self._red = list(map_refs), list(reduce_refs)
        self.num_map, self.num_reduce = len(self._map), len(self._red)
        self.map_done = self.reduce_done = 0

    def poll(self):
        if self._map:
            ready, self._map = _w.wait(self._map, num_returns=len(self._map), timeout=0)
            self.map_done += len(ready)
        if self._red:
            ready, self._red = _w.wait(self._red, num_returns=len(self._red), timeout=0)
            self.reduce_done += len(ready)
        return self.map_done, self.reduce_done


def simple_shuffle(*, input_reader: Callable[[PartitionID], Iterable[Any]], input_num_partitions: int,
                   output_num_partitions: int, output_writer: Callable[[PartitionID, List[Any]], Any],
                   partitioner: Callable = round_robin_partitioner, object_store_writer=ObjectStoreWriter,
                   map_options: Optional[dict] = None, reduce_options: Optional[dict] = None,
                   progress: Optional[Callable[[ShuffleProgress], None]] = None) -> List[Any]:
    """Shuffle ``input_num_partitions`` inputs into ``output_num_partitions`` outputs; returns the
    output writers' results in partition order. ``output_writer(j, items)`` receives, for a
    streaming ``object_store_writer`` (the default), the object refs of partition j's items (fetch
    them with ``ray.get`` / ``ray.wait``), else the items. ``progress``: called with a
    ``ShuffleProgress`` about every 0.2 s until the reduces finish."""
    from .. import remote

    if input_num_partitions < 1 or output_num_partitions < 1:
        raise ValueError("partition counts must be >= 1")
    streaming = object_store_writer is not ObjectStoreWriterNonStreaming and not issubclass(
        object_store_writer, ObjectStoreWriterNonStreaming)
    map_task = remote(num_returns=output_num_partitions, **(map_options or {}))(_map)
    reduce_task = remote(**(reduce_options or {}))(_reduce)
    map_out = []
    for i in range(input_num_partitions):
        refs = map_task.remote(input_reader, partitioner, object_store_writer, output_num_partitions, i)
        map_out.append(refs if output_num_partitions > 1 else [refs])
    reduce_refs = [reduce_task.remote(output_writer, streaming, j, *[m[j] for m in map_out])
                   for j in range(output_num_partitions)]
    if progress is not None:
        tracker = ShuffleProgress([r for m in map_out for r in m], reduce_refs)
        while tracker.poll()[1] < tracker.num_reduce:
            progress(tracker)
            time.sleep(0.2)
        progress(tracker)
    return _w.get(reduce_refs)


def run(num_partitions: int = 5, partition_size: float = 200e6, num_nodes: Optional[int] = None,
        num_cpus: int = 8, object_store_memory: float = 1e9, ray_address: Optional[str] = None,
        no_streaming: bool = False, use_wait: bool = False) -> dict:
    """The reference's shuffle driver: ``num_partitions`` x ``num_partitions`` shuffle of
    ``partition_size``-byte uint8 partitions, each split into 1 MB-ish rows (``rows_per_partition``
    = max(1, size / 1e6)). Returns the statistics it prints."""
    from .. import cluster_utils

    cluster = None
    started = False
    if ray_address:
        _w.init(address=ray_address, ignore_reinit_error=True)
    elif num_nodes:  # virtual nodes of one session (the first add_node starts it)
        cluster = cluster_utils.Cluster()
        for _ in range(num_nodes):
            cluster.add_node(num_cpus=num_cpus, object_store_memory=int(object_store_memory))
    elif not _w.is_initialized():
        _w.init(num_cpus=num_cpus, object_store_memory=int(object_store_memory))
        started = True
    rows = max(1, int(partition_size // 1_000_000))
    row_bytes = int(partition_size // rows)

    def input_reader(i):
        for _ in range(rows):
            yield np.ones(row_bytes, dtype=np.uint8)

    def output_writer(j, items):
        total = 0
        if no_streaming:
            return int(sum(int(a.size) for a in items))
        if use_wait:
            pending = list(items)
            while pending:
                [ready], pending = _w.wait(pending, num_returns=1)
                total += int(_w.get(ready).size)
        else:
            for ref in items:
                total += int(_w.get(ref).size)
        return total

    t0 = time.time()
    out = simple_shuffle(input_reader=input_reader, input_num_partitions=num_partitions,
                         output_num_partitions=num_partitions, output_writer=output_writer,
                         object_store_writer=ObjectStoreWriterNonStreaming if no_streaming else ObjectStoreWriter)
    dt = time.time() - t0
    total = int(sum(out))
    stats = {"shuffled_bytes": total, "seconds": round(dt, 3), "mb_per_s": round(total / 1e6 / max(dt, 1e-9), 1),
             "num_partitions": num_partitions, "partition_size": int(partition_size)}
    try:
        stats["object_store"] = _w._core().client.call("store_stats")
    except Exception:  # noqa - stats are best effort
        pass
    if cluster is not None:
        cluster.shutdown()
    elif started:
        _w.shutdown()
    return stats


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ray-address", default=None)
    ap.add_argument("--object-store-memory", type=float, default=1e9)
    ap.add_argument("--num-partitions", type=int, default=5)
    ap.add_argument("--partition-size", type=float, default=200e6)
    ap.add_argument("--num-nodes", type=int, default=None)
    ap.add_argument("--num-cpus", type=int, default=8)
    ap.add_argument("--no-streaming", action="store_true")
    ap.add_argument("--use-wait", action="store_true")
    a = ap.parse_args(argv)
    stats = run(a.num_partitions, a.partition_size, a.num_nodes, a.num_cpus, a.object_store_memory, a.ray_address,
                a.no_streaming, a.use_wait)
    print(f"Shuffled {stats['shuffled_bytes'] / 2**20:.0f} MiB in {stats['seconds']} seconds")
    print(json.dumps(stats, default=str))


if __name__ == "__main__":
    main()
