"""``ray.tune.syncer`` (reference: python/ray/tune/syncer.py). Experiment and trial directories
live on the (shared or local) storage path directly, so there is nothing to upload: ``SyncConfig``
is accepted for its options and ``Syncer`` implements ``sync_up`` / ``sync_down`` / ``delete`` as
local directory copies, for storage paths that need an explicit mirror."""
from __future__ import annotations

import os
import shutil
from typing import List, Optional

from ..air.config import SyncConfig


class Syncer:
    def __init__(self, sync_period: float = 300.0, sync_timeout: float = 1800.0):
        self.sync_period, self.sync_timeout = sync_period, sync_timeout

    def sync_up(self, local_dir: str, remote_dir: str, exclude: Optional[List[str]] = None) -> bool:
        shutil.copytree(local_dir, remote_dir, dirs_exist_ok=True,
                        ignore=shutil.ignore_patterns(*exclude) if exclude else None)
        return True

    def sync_down(self, remote_dir: str, local_dir: str, exclude: Optional[List[str]] = None) -> bool:
        return self.sync_up(remote_dir, local_dir, exclude)

    def delete(self, remote_dir: str) -> bool:
        shutil.rmtree(remote_dir, ignore_errors=True)
        return not os.path.exists(remote_dir)

    def wait(self) -> None:
        pass


__all__ = ["SyncConfig", "Syncer"]
