"""EnvContext: the ``env_config`` dict an env creator receives, plus where it runs (reference:
rllib/env/env_context.py). Env creators registered with ``register_env`` get one, so an env can
seed or shard itself by ``worker_index`` / ``vector_index``."""
from __future__ import annotations

import copy
from typing import Optional


class EnvContext(dict):
    def __init__(self, env_config: Optional[dict] = None, worker_index: int = 0, vector_index: int = 0,
                 remote: bool = False, num_workers: Optional[int] = None, recreated_worker: bool = False):
        super().__init__(env_config or {})
        self.worker_index = worker_index
        self.vector_index = vector_index
        self.remote = remote
        self.num_workers = num_workers
        self.recreated_worker = recreated_worker

    def copy_with_overrides(self, env_config: Optional[dict] = None, worker_index: Optional[int] = None,
                            vector_index: Optional[int] = None, remote: Optional[bool] = None,
                            num_workers: Optional[int] = None,
                            recreated_worker: Optional[bool] = None) -> "EnvContext":
        return EnvContext(copy.deepcopy(env_config) if env_config is not None else dict(self),
                          self.worker_index if worker_index is None else worker_index,
                          self.vector_index if vector_index is None else vector_index,
                          self.remote if remote is None else remote,
                          self.num_workers if num_workers is None else num_workers,
                          self.recreated_worker if recreated_worker is None else recreated_worker)

    def set_defaults(self, defaults: dict) -> None:
        for k, v in defaults.items():
            self.setdefault(k, v)

    def __str__(self):
        return (f"{dict.__repr__(self)[:-1]}, worker={self.worker_index}/{self.num_workers}, "
                f"vector_idx={self.vector_index}, remote={self.remote}}}")
