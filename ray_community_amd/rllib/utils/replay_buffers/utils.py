"""Replay-buffer helpers (reference: rllib/utils/replay_buffers/utils.py)."""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np


def update_priorities_in_replay_buffer(replay_buffer, config: Dict, train_batch, train_results: Dict) -> None:
    """Push the learner's TD errors back into a prioritized buffer: per policy,
    ``train_results[pid]["td_error"]`` against ``train_batch[pid]["batch_indexes"]``."""
    if not hasattr(replay_buffer, "update_priorities"):
        return
    prio = {}
    for pid, res in (train_results or {}).items():
        td = (res or {}).get("td_error")
        if td is None:
            continue
        batch = train_batch[pid] if hasattr(train_batch, "policy_batches") else train_batch
        idx = batch.get("batch_indexes") if hasattr(batch, "get") else None
        if idx is not None:
            prio[pid] = (np.asarray(idx), np.asarray(td))
    if prio:
        replay_buffer.update_priorities(prio)


def sample_min_n_steps_from_buffer(replay_buffer, min_steps: int, count_by_agent_steps: bool = False) -> Optional[object]:
    """Sample until at least ``min_steps`` rows (None from an empty buffer)."""
    if len(replay_buffer) == 0:
        return None
    return replay_buffer.sample(int(min_steps))
