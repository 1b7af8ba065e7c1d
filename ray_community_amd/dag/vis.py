"""DAG visualisation (reference ``python/ray/dag/vis_utils.py::plot``): the graph is rendered as
Graphviz DOT text. ``to_file`` ending in ``.dot`` gets the text; other suffixes (``.png``, ``.svg``)
are rendered by the ``dot`` binary when it is installed."""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import Optional

from .dag_node import DAGNode


def _label(node: DAGNode) -> str:
    cls = type(node).__name__
    for attr in ("_body", "_remote_function", "_method_name", "_key"):
        v = getattr(node, attr, None)
        if v is not None:
            name = getattr(v, "_name", None) or getattr(v, "__name__", None) or str(v)
            return f"{cls}\\n{name}"
    return cls


def to_dot(dag: DAGNode) -> str:
    ids, lines, stack, seen = {}, [], [dag], set()
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        ids.setdefault(id(n), f"n{len(ids)}")
        lines.append(f'  {ids[id(n)]} [label="{_label(n)}"];')
        for c in n._children():
            ids.setdefault(id(c), f"n{len(ids)}")
            lines.append(f"  {ids[id(c)]} -> {ids[id(n)]};")
            stack.append(c)
    return "digraph DAG {\n  rankdir=LR;\n" + "\n".join(lines) + "\n}\n"


def plot(dag: DAGNode, to_file: Optional[str] = None) -> str:
    """Write the DAG to ``to_file`` (default ``ray_dag.dot``); returns the path written."""
    to_file = to_file or "ray_dag.dot"
    text = to_dot(dag)
    ext = os.path.splitext(to_file)[1].lstrip(".").lower()
    if ext in ("", "dot", "gv"):
        with open(to_file, "w") as f:
            f.write(text)
        return to_file
    exe = shutil.which("dot")
    if exe is None:
        raise ImportError("rendering to ." + ext + " needs the graphviz 'dot' binary; use a .dot file name")
    subprocess.run([exe, "-T" + ext, "-o", to_file], input=text.encode(), check=True)
    return to_file
