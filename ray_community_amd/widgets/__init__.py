"""Notebook display helpers (reference ``python/ray/widgets``): HTML templates for objects'
``_repr_html_`` and a dict -> HTML table helper. Plain-string rendering (no ipywidgets needed)."""
from __future__ import annotations

import html
from typing import Any, Dict


class Template:
    """A tiny ``{{ name }}`` substitution template (reference ``ray.widgets.Template`` loads its
    templates from files; here the text is given directly)."""

    def __init__(self, text: str):
        self.text = text

    def render(self, **kwargs) -> str:
        out = self.text
        for k, v in kwargs.items():
            out = out.replace("{{ " + k + " }}", str(v)).replace("{{" + k + "}}", str(v))
        return out


def make_table_html_repr(obj: Any, title: str = "", max_height: str = "none") -> str:
    """An HTML table of ``obj``'s public attributes (or of a dict), for ``_repr_html_``."""
    items: Dict[str, Any] = obj if isinstance(obj, dict) else {
        k: v for k, v in vars(obj).items() if not k.startswith("_")}
    rows = "".join(f"<tr><td>{html.escape(str(k))}</td><td>{html.escape(str(v))}</td></tr>" for k, v in items.items())
    head = f"<h3>{html.escape(title)}</h3>" if title else ""
    return f'<div style="max-height:{max_height};overflow:auto">{head}<table>{rows}</table></div>'


__all__ = ["Template", "make_table_html_repr"]
