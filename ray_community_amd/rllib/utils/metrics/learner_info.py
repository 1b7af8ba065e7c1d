"""Aggregating learner results over minibatches / towers (reference:
rllib/utils/metrics/learner_info.py): ``add_learn_on_batch_results(results, policy_id)`` per
update, ``finalize()`` -> ``{policy_id: {stat: mean over the updates}}`` (non-numeric values
keep the last one)."""
from __future__ import annotations

import collections
from typing import Dict

import numpy as np

from . import ALL_MODULES, LEARNER_INFO, LEARNER_STATS_KEY  # noqa: F401


class LearnerInfoBuilder:
    def __init__(self, num_devices: int = 1):
        self.num_devices = num_devices
        self.results_all_towers: Dict[str, list] = collections.defaultdict(list)
        self.is_finalized = False

    def add_learn_on_batch_results(self, results: Dict, policy_id: str = "default_policy") -> None:
        if self.is_finalized:
            raise AssertionError("LearnerInfoBuilder already finalized")
        self.results_all_towers[policy_id].append(results)

    def add_learn_on_batch_results_multi_agent(self, all_policies_results: Dict) -> None:
        for pid, res in all_policies_results.items():
            self.add_learn_on_batch_results(res, pid)

    def finalize(self) -> Dict:
        self.is_finalized = True
        out = {}
        for pid, rs in self.results_all_towers.items():
            out[pid] = _reduce(rs)
        return out


def _reduce(dicts):
    out = {}
    keys = {k for d in dicts for k in d}
    for k in keys:
        vals = [d[k] for d in dicts if k in d]
        if all(isinstance(v, dict) for v in vals):
            out[k] = _reduce(vals)
        elif all(isinstance(v, (int, float, np.number)) and not isinstance(v, bool) for v in vals):
            out[k] = float(np.mean(vals))
        else:
            out[k] = vals[-1]
    return out
