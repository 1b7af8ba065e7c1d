"""Old-API-stack evaluation names (reference: rllib/evaluation/__init__.py).

``RolloutWorker`` is this framework's ``EnvRunner``; ``SampleBatchBuilder`` /
``MultiAgentSampleBatchBuilder`` collect rows into (multi-agent) batches; ``SyncSampler`` pulls
fragments from a runner; ``collect_metrics`` summarises the episodes runners finished."""
from __future__ import annotations

import collections
from typing import Any, Dict, Iterable, List, Optional

import numpy as np

from ..algorithms.callbacks import Episode
from ..env.env_runner import EnvRunner
from ..policy.sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch
from .postprocessing import compute_advantages

RolloutWorker = EnvRunner


class SampleBatchBuilder:
    """Row-wise accumulation: ``add_values(**row)`` then ``build_and_reset()``."""

    def __init__(self):
        self.buffers: Dict[str, List[Any]] = collections.defaultdict(list)
        self.count = 0

    def add_values(self, **values) -> None:
        for k, v in values.items():
            self.buffers[k].append(v)
        self.count += 1

    def add_batch(self, batch: SampleBatch) -> None:
        for k, v in batch.items():
            self.buffers[k].extend(list(v))
        self.count += batch.count

    def build_and_reset(self) -> SampleBatch:
        b = SampleBatch({k: np.asarray(v) for k, v in self.buffers.items()})
        self.buffers = collections.defaultdict(list)
        self.count = 0
        return b


class MultiAgentSampleBatchBuilder:
    """Per-agent builders; ``postprocess_batch_so_far`` moves each agent's rows (through its
    policy's ``postprocess_trajectory`` if it has one) into per-policy builders, and
    ``build_and_reset`` returns the MultiAgentBatch."""

    def __init__(self, policy_map: Optional[Dict[str, Any]] = None, clip_rewards: bool = False, callbacks=None):
        self.policy_map = dict(policy_map or {})
        self.clip_rewards = clip_rewards
        self.callbacks = callbacks
        self.agent_builders: Dict[Any, SampleBatchBuilder] = {}
        self.agent_to_policy: Dict[Any, str] = {}
        self.policy_builders: Dict[str, SampleBatchBuilder] = collections.defaultdict(SampleBatchBuilder)
        self.count = 0

    def total(self) -> int:
        return sum(b.count for b in self.agent_builders.values())

    def has_pending_agent_data(self) -> bool:
        return any(b.count for b in self.agent_builders.values())

    def add_values(self, agent_id, policy_id: str = DEFAULT_POLICY_ID, **values) -> None:
        self.agent_to_policy[agent_id] = policy_id
        self.agent_builders.setdefault(agent_id, SampleBatchBuilder()).add_values(**values)

    def count_steps(self) -> None:
        self.count += 1

    def postprocess_batch_so_far(self, episode=None) -> None:
        for aid, builder in list(self.agent_builders.items()):
            if not builder.count:
                continue
            batch = builder.build_and_reset()
            if self.clip_rewards and SampleBatch.REWARDS in batch:
                batch[SampleBatch.REWARDS] = np.sign(batch[SampleBatch.REWARDS])
            pid = self.agent_to_policy[aid]
            pol = self.policy_map.get(pid)
            if pol is not None and hasattr(pol, "postprocess_trajectory"):
                batch = pol.postprocess_trajectory(batch)
            self.policy_builders[pid].add_batch(batch)

    def build_and_reset(self, episode=None) -> MultiAgentBatch:
        self.postprocess_batch_so_far(episode)
        out = {pid: b.build_and_reset() for pid, b in self.policy_builders.items() if b.count}
        n = self.count or max((b.count for b in out.values()), default=0)
        self.policy_builders = collections.defaultdict(SampleBatchBuilder)
        self.count = 0
        return MultiAgentBatch(out, n)


class SyncSampler:
    """Synchronous sampling from one env runner: ``get_data()`` -> one rollout fragment."""

    def __init__(self, env_runner=None, *, worker=None, rollout_fragment_length: Optional[int] = None, **kw):
        self.runner = env_runner if env_runner is not None else worker
        self.rollout_fragment_length = rollout_fragment_length

    def get_data(self) -> SampleBatch:
        return self.runner.sample(self.rollout_fragment_length)

    def get_metrics(self) -> List[Dict]:
        return [self.runner.get_metrics()]

    def get_extra_batches(self) -> List[SampleBatch]:
        return []


def summarize_episodes(episodes: Iterable, new_episodes: Optional[Iterable] = None,
                       keep_custom_metrics: bool = False) -> Dict:
    eps = list(episodes)
    rets = [float(e[0]) for e in eps]
    lens = [int(e[1]) for e in eps]
    nan = float("nan")
    return {"episode_reward_mean": float(np.mean(rets)) if rets else nan,
            "episode_reward_max": float(np.max(rets)) if rets else nan,
            "episode_reward_min": float(np.min(rets)) if rets else nan,
            "episode_len_mean": float(np.mean(lens)) if lens else nan,
            "episodes_this_iter": len(list(new_episodes)) if new_episodes is not None else len(eps),
            "hist_stats": {"episode_reward": rets, "episode_lengths": lens}}


def collect_episodes(runners: Iterable, timeout_seconds: float = 180) -> List:
    """``(return, length)`` of the episodes each runner (local object or actor handle) finished
    since it was last asked."""
    from ... import get

    eps = []
    for r in runners:
        m = get(r.get_metrics.remote(), timeout=timeout_seconds) if hasattr(r, "get_metrics") and \
            hasattr(r.get_metrics, "remote") else r.get_metrics()
        eps.extend(m.get("episodes", []))
    return eps


def collect_metrics(workers=None, remote_worker_ids=None, timeout_seconds: float = 180,
                    keep_custom_metrics: bool = False) -> Dict:
    """Episode summary over ``workers`` (an EnvRunnerGroup or a list of runners)."""
    if workers is None:
        return summarize_episodes([])
    if hasattr(workers, "healthy_env_runners"):
        local = workers.local_env_runner()
        runners = ([local] if local is not None else []) + list(workers.healthy_env_runners())
    else:
        runners = list(workers)
    return summarize_episodes(collect_episodes(runners, timeout_seconds))


__all__ = ["RolloutWorker", "SampleBatch", "MultiAgentBatch", "SampleBatchBuilder", "MultiAgentSampleBatchBuilder",
           "SyncSampler", "compute_advantages", "collect_metrics", "collect_episodes", "summarize_episodes", "Episode"]
