"""Worker stdout/stderr -> driver forwarding (``ray.init(log_to_driver=True)``) and log-file access.

Reference behaviour: ``python/ray/_private/log_monitor.py`` tails every worker's log files on a
node and publishes new lines through GCS pubsub; the driver's ``print_worker_logs``
(``_private/worker.py``) prints them as ``(TaskOrActorName pid=1234) line``, filtered to its job.

Here every worker process writes stdout+stderr (unbuffered, ``python -u``) into
``<session>/logs/worker-<id>.out``. One monitor thread in the head polls the files it knows about,
reads only the bytes appended since its last pass (``os.pread`` at the saved offset, bounded per
pass), splits complete lines (a trailing partial line waits for its newline), tags each batch with
the worker's pid and what it runs (actor class / last task name) and hands it to every sink: the
in-process driver prints it, socket drivers that registered with ``log_to_driver`` receive one
``LOG_BATCH`` frame per pass. A dead worker's file is drained one last time before it is dropped.
"""
from __future__ import annotations

import os
import sys
import threading
from typing import Callable, Dict, List, Optional

MAX_READ_PER_FILE = 1 << 20  # bytes per file per pass: a chatty worker cannot stall the others
# a worker writes "<MARK><label>" on a line of its own before running a task of another name (and
# once when it becomes an actor): the monitor takes the label for the lines that follow and drops
# the marker line (the reference's ":task_name:" / ":actor_name:" lines, log_monitor.py)
LOG_LABEL_MARK = "::rca-label::"
_MARK_B = LOG_LABEL_MARK.encode()


class _Tail:
    __slots__ = ("path", "offset", "partial", "pid", "label", "node", "gone")

    def __init__(self, path, pid, label, node, offset=0):
        self.path = path
        self.offset = offset
        self.partial = b""
        self.pid = pid
        self.label = label
        self.node = node
        self.gone = False


def format_batch(batch: dict) -> List[str]:
    """Driver-side rendering, reference style: ``(Label pid=123) text`` (``(pid=123)`` without a label)."""
    label = batch.get("label")
    head = f"({label} pid={batch['pid']})" if label else f"(pid={batch['pid']})"
    if batch.get("node") and batch.get("remote_node"):
        head = head[:-1] + f", node={batch['node'][:8]})"
    return [f"{head} {ln}" for ln in batch["lines"]]


def print_batches(batches, stream=None):
    out = stream or sys.stdout
    try:
        for b in batches:
            for line in format_batch(b):
                print(line, file=out)
        out.flush()
    except Exception:  # noqa  (a closed driver stdout must not kill the monitor)
        pass


class LogMonitor:
    """Polls worker log files for the head. ``describe()`` (called under the head lock) returns
    ``{worker_id: (path, pid, label, node_id, alive)}`` for the workers that exist now."""

    def __init__(self, describe: Callable[[], Dict[bytes, tuple]], lock, interval_s: float = 0.1):
        self.describe = describe
        self.lock = lock
        self.interval_s = interval_s
        self.sinks: List[Callable[[list], None]] = []
        self._tails: Dict[bytes, _Tail] = {}
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._poll_lock = threading.Lock()

    def add_sink(self, fn):
        self.sinks.append(fn)

    def remove_sink(self, fn):
        try:
            self.sinks.remove(fn)
        except ValueError:
            pass

    def start(self):
        self._thread = threading.Thread(target=self._run, name="rca-log-monitor", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
        self.poll()  # last lines of workers that exited during shutdown

    def _run(self):
        while not self._stop.wait(self.interval_s):
            try:
                self.poll()
            except Exception:  # noqa
                pass

    def poll(self) -> list:
        with self._poll_lock:
            with self.lock:
                live = self.describe()
            for wid, (path, pid, label, node, _alive) in live.items():
                t = self._tails.get(wid)
                if t is None:
                    self._tails[wid] = _Tail(path, pid, label, node)
                else:
                    t.pid = pid or t.pid
                    if label:
                        t.label = label
            for wid, t in self._tails.items():
                if wid not in live:
                    t.gone = True
            batches = []
            for wid in list(self._tails):
                t = self._tails[wid]
                cur = []
                for raw in self._read(t):
                    if raw.startswith(_MARK_B):
                        if cur:
                            batches.append({"pid": t.pid, "label": t.label, "node": t.node, "lines": cur})
                            cur = []
                        t.label = raw[len(_MARK_B):].decode("utf-8", "replace") or t.label
                        continue
                    cur.append(raw.decode("utf-8", "replace"))
                if cur:
                    batches.append({"pid": t.pid, "label": t.label, "node": t.node, "lines": cur})
                if t.gone:
                    del self._tails[wid]
            if batches:
                for s in list(self.sinks):
                    try:
                        s(batches)
                    except Exception:  # noqa
                        pass
            return batches

    @staticmethod
    def _read(t: _Tail) -> List[bytes]:
        try:
            fd = os.open(t.path, os.O_RDONLY)
        except OSError:
            return []
        try:
            data = os.pread(fd, MAX_READ_PER_FILE, t.offset)
        except OSError:
            data = b""
        finally:
            os.close(fd)
        if not data:
            if t.gone and t.partial:  # process ended without a final newline
                last, t.partial = t.partial, b""
                return [last]
            return []
        t.offset += len(data)
        data = t.partial + data
        cut = data.rfind(b"\n")
        if cut < 0:
            t.partial = data
            return []
        t.partial = data[cut + 1:]
        return data[:cut].split(b"\n")


def read_log(path: str, tail: int = -1, max_bytes: int = 64 << 20) -> List[str]:
    """Lines of one log file; ``tail`` > 0 keeps only the last ``tail`` lines."""
    try:
        size = os.path.getsize(path)
        with open(path, "rb") as f:
            if size > max_bytes:
                f.seek(size - max_bytes)
            data = f.read()
    except OSError:
        return []
    lines = [ln for ln in data.decode("utf-8", "replace").splitlines() if not ln.startswith(LOG_LABEL_MARK)]
    return lines[-tail:] if tail and tail > 0 else lines
