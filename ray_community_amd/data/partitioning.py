"""Path-based partitioning of file datasets (reference: python/ray/data/datasource/partitioning.py,
file_based_datasource.py:FileExtensionFilter).

* ``Partitioning(style, base_dir, field_names, field_types)``: HIVE (``col=value`` directories) or
  DIRECTORY (positional directories named by ``field_names``).
* ``PathPartitionParser(partitioning)(path) -> {field: value}``; values are strings unless
  ``field_types`` maps a field to a type (``int``, ``float``, ...).
* ``PathPartitionFilter.of(filter_fn, style=..., ...)(paths) -> kept paths``: prune files by
  their partition values before any read task is created (``read_*(partition_filter=...)``).
"""
from __future__ import annotations

import os
import posixpath
from dataclasses import dataclass
from enum import Enum
from typing import Callable, Dict, List, Optional, Union


class PartitionStyle(str, Enum):
    HIVE = "hive"
    DIRECTORY = "dir"

    def __str__(self):
        return self.value


@dataclass
class Partitioning:
    style: Union[PartitionStyle, str] = PartitionStyle.HIVE
    base_dir: Optional[str] = None
    field_names: Optional[List[str]] = None
    field_types: Optional[Dict[str, type]] = None
    filesystem: object = None

    def __post_init__(self):
        self.style = PartitionStyle(str(getattr(self.style, "value", self.style)).lower())
        if self.style == PartitionStyle.DIRECTORY and not self.field_names:
            raise ValueError("DIRECTORY partitioning needs field_names (one per directory level)")
        self.base_dir = self.base_dir or ""
        self.field_types = dict(self.field_types or {})

    @property
    def normalized_base_dir(self) -> str:
        b = self.base_dir.rstrip("/\\")
        return b + "/" if b else ""


def _rel_dirs(path: str, base: str) -> List[str]:
    """Directory components of ``path`` below ``base`` (all of them when ``base`` is empty)."""
    d = os.path.dirname(os.path.normpath(path))
    if base:
        rel = os.path.relpath(d, os.path.normpath(base))
        if rel.startswith(".."):
            raise ValueError(f"{path!r} is not under the partitioning base directory {base!r}")
    else:
        rel = d
    return [p for p in rel.replace("\\", "/").split("/") if p not in ("", ".")]


class PathPartitionParser:
    """Partition field values from one file path."""

    def __init__(self, partitioning: Partitioning):
        self._p = partitioning

    @classmethod
    def of(cls, style: Union[PartitionStyle, str] = PartitionStyle.HIVE, base_dir: Optional[str] = None,
           field_names: Optional[List[str]] = None, field_types: Optional[Dict[str, type]] = None,
           filesystem=None) -> "PathPartitionParser":
        return cls(Partitioning(style, base_dir, field_names, field_types, filesystem))

    @property
    def scheme(self) -> Partitioning:
        return self._p

    def _cast(self, out: Dict[str, str]) -> Dict[str, object]:
        for k, t in self._p.field_types.items():
            if k in out:
                out[k] = t(out[k])
        return out

    def __call__(self, path: str) -> Dict[str, object]:
        dirs = _rel_dirs(path, self._p.base_dir)
        if self._p.style == PartitionStyle.HIVE:
            out = {}
            for part in dirs:
                if "=" in part:
                    k, v = part.split("=", 1)
                    out[k] = v
            if self._p.field_names:
                missing = [f for f in self._p.field_names if f not in out]
                if missing:
                    raise ValueError(f"{path!r} lacks HIVE partition fields {missing}")
            return self._cast(out)
        names = self._p.field_names
        if len(dirs) < len(names):  # the partition directories are the LAST len(names) levels
            raise ValueError(f"{path!r} has {len(dirs)} directory levels, expected {len(names)} ({names})")
        return self._cast(dict(zip(names, dirs[len(dirs) - len(names):])))


class PathPartitionFilter:
    """Keep the paths whose partition values pass ``filter_fn(values) -> bool``."""

    def __init__(self, path_partition_parser: PathPartitionParser, filter_fn: Callable[[Dict[str, str]], bool]):
        self._parser = path_partition_parser
        self._fn = filter_fn

    @classmethod
    def of(cls, filter_fn: Callable[[Dict[str, str]], bool], style: Union[PartitionStyle, str] = PartitionStyle.HIVE,
           base_dir: Optional[str] = None, field_names: Optional[List[str]] = None,
           field_types: Optional[Dict[str, type]] = None, filesystem=None) -> "PathPartitionFilter":
        return cls(PathPartitionParser.of(style, base_dir, field_names, field_types, filesystem), filter_fn)

    @property
    def parser(self) -> PathPartitionParser:
        return self._parser

    def __call__(self, paths: List[str]) -> List[str]:
        out = []
        for p in paths:
            try:
                vals = self._parser(p)
            except ValueError:
                continue  # not a partition file of this scheme
            if vals and self._fn(vals):
                out.append(p)
        return out


class FileExtensionFilter:
    """Keep paths with one of ``file_extensions`` (case-insensitive); files without an extension
    pass when ``allow_if_no_extension``."""

    def __init__(self, file_extensions: Union[str, List[str]], allow_if_no_extension: bool = False):
        exts = [file_extensions] if isinstance(file_extensions, str) else list(file_extensions)
        self.extensions = [e.lower().lstrip(".") for e in exts]
        self.allow_if_no_extension = allow_if_no_extension

    def _ok(self, path: str) -> bool:
        ext = posixpath.splitext(path.replace("\\", "/"))[1].lower().lstrip(".")
        if not ext:
            return self.allow_if_no_extension
        return ext in self.extensions

    def __call__(self, paths: List[str]) -> List[str]:
        return [p for p in paths if self._ok(p)]


__all__ = ["PartitionStyle", "Partitioning", "PathPartitionParser", "PathPartitionFilter", "FileExtensionFilter"]
