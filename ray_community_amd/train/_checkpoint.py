"""Directory-based checkpoints (reference: ``python/ray/train/_checkpoint.py``)."""
from __future__ import annotations

import contextlib
import json
import os
import shutil
import tempfile
import uuid
from typing import Any, Dict, Iterator, Optional

_METADATA_FILE = ".metadata.json"


class Checkpoint:
    """A reference to a directory of checkpoint files (local filesystem)."""

    def __init__(self, path: str, filesystem=None):
        self.path = os.fspath(path)
        self.filesystem = filesystem
        self._uuid = uuid.uuid4()

    @classmethod
    def from_directory(cls, path) -> "Checkpoint":
        return cls(os.path.abspath(os.fspath(path)))

    def to_directory(self, path: Optional[str] = None) -> str:
        dst = os.fspath(path) if path is not None else tempfile.mkdtemp(prefix="checkpoint_")
        os.makedirs(dst, exist_ok=True)
        if os.path.abspath(dst) != os.path.abspath(self.path):
            shutil.copytree(self.path, dst, dirs_exist_ok=True)
        return dst

    @contextlib.contextmanager
    def as_directory(self) -> Iterator[str]:
        yield self.path

    def get_metadata(self) -> Dict[str, Any]:
        p = os.path.join(self.path, _METADATA_FILE)
        if not os.path.exists(p):
            return {}
        with open(p) as f:
            return json.load(f)

    def set_metadata(self, metadata: Dict[str, Any]):
        with open(os.path.join(self.path, _METADATA_FILE), "w") as f:
            json.dump(metadata, f)

    def update_metadata(self, metadata: Dict[str, Any]):
        m = self.get_metadata()
        m.update(metadata)
        self.set_metadata(m)

    def __repr__(self):
        return f"Checkpoint(filesystem=local, path={self.path})"

    def __eq__(self, other):
        return isinstance(other, Checkpoint) and other.path == self.path

    def __hash__(self):
        return hash(self.path)

    def __fspath__(self):
        return self.path
