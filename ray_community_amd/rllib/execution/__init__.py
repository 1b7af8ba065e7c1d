"""Old-API-stack execution helpers (reference: rllib/execution/{rollout_ops,train_ops,
learner_thread,multi_gpu_learner_thread,minibatch_buffer,replay_ops}.py), written against this
framework's EnvRunnerGroup / LearnerGroup so custom ``training_step`` code composes the same way:

    batch = synchronous_parallel_sample(worker_set=algo.env_runner_group, max_env_steps=4000)
    batch = standardize_fields(batch, ["advantages"])
    results = train_one_step(algo, batch)
"""
from __future__ import annotations

import queue
import random
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np

from ..policy.sample_batch import MultiAgentBatch, SampleBatch, concat_samples


def synchronous_parallel_sample(*, worker_set, max_agent_steps: Optional[int] = None,
                                max_env_steps: Optional[int] = None, concat: bool = True,
                                sample_timeout_s: Optional[float] = None, **kw):
    """Sample from every healthy remote env runner (the local one if there are none) in rounds
    until ``max_env_steps`` (or ``max_agent_steps``) are collected; one round if neither is set."""
    target = max_env_steps or max_agent_steps
    got: List[Any] = []
    steps = 0
    while True:
        if worker_set.num_healthy_remote_env_runners() > 0:
            round_ = worker_set.foreach_env_runner("sample", timeout_seconds=sample_timeout_s)
        else:
            round_ = [worker_set.local_env_runner().sample()]
        for b in round_:
            got.append(b)
            steps += b.agent_steps() if (max_agent_steps and hasattr(b, "agent_steps")) else len(b)
        if not target or steps >= target or not round_:
            break
    if not concat:
        return got
    if got and isinstance(got[0], MultiAgentBatch):
        pids = {p for b in got for p in b.policy_batches}
        return MultiAgentBatch({p: concat_samples([b.policy_batches[p] for b in got if p in b.policy_batches])
                                for p in pids}, sum(len(b) for b in got))
    return concat_samples(got) if got else SampleBatch({})


def standardize_fields(samples, fields: List[str]):
    """Zero-mean / unit-std the given columns (per policy for a MultiAgentBatch), in place."""
    batches = samples.policy_batches.values() if isinstance(samples, MultiAgentBatch) else [samples]
    for b in batches:
        for f in fields:
            if f in b:
                v = np.asarray(b[f], dtype=np.float32)
                b[f] = (v - v.mean()) / max(1e-4, float(v.std()))
    return samples


_KINDS = ("ppo", "impala", "appo", "dqn", "marwil", "sac", "cql")


def _update_kind(algorithm) -> str:
    """The Learner update the algorithm trains with: its ``_update_kind``, else the first class in
    its MRO with a Learner update of that name (BC -> MARWIL's)."""
    kind = getattr(algorithm, "_update_kind", None)
    if kind:
        return kind
    for cls in type(algorithm).__mro__:
        if cls.__name__.lower() in _KINDS:
            return cls.__name__.lower()
    raise ValueError(f"no Learner update for {type(algorithm).__name__}; pass a PPO/IMPALA/APPO/DQN/"
                     f"MARWIL/BC/SAC/CQL algorithm")


def train_one_step(algorithm, train_batch, policies_to_train: Optional[List[str]] = None) -> Dict:
    """One learner update on ``train_batch`` through the algorithm's LearnerGroup(s); per-policy
    results for a MultiAgentBatch."""
    kind = _update_kind(algorithm)
    if isinstance(train_batch, MultiAgentBatch) and getattr(algorithm, "learner_groups", None):
        out = {}
        for pid, b in train_batch.policy_batches.items():
            if policies_to_train is None or pid in policies_to_train:
                out[pid] = algorithm.learner_groups[pid].update(kind, b)
        return out
    return {"default_policy": algorithm.learner_group.update(kind, train_batch)}


multi_gpu_train_one_step = train_one_step  # the LearnerGroup already spreads a batch over its GPUs


class SimpleReplayBuffer:
    """Keeps the last ``num_slots`` batches and replays a random one."""

    def __init__(self, num_slots: int, replay_proportion: Optional[float] = None):
        self.num_slots = int(num_slots)
        self.replay_batches: List[Any] = []
        self.replay_index = 0

    def add_batch(self, sample_batch) -> None:
        if self.num_slots <= 0:
            return
        if len(self.replay_batches) < self.num_slots:
            self.replay_batches.append(sample_batch)
        else:
            self.replay_batches[self.replay_index] = sample_batch
            self.replay_index = (self.replay_index + 1) % self.num_slots

    def replay(self):
        return random.choice(self.replay_batches)

    def __len__(self):
        return len(self.replay_batches)


class MinibatchBuffer:
    """Hands each batch from ``inqueue`` out ``num_passes`` times (``init_num_passes`` for the
    first one); ``get()`` -> (batch, released) where released says the batch is done."""

    def __init__(self, inqueue: "queue.Queue", size: int, timeout: float, num_passes: int,
                 init_num_passes: int = 1):
        self.inqueue, self.size, self.timeout = inqueue, int(size), timeout
        self.max_ttl, self.cur_max_ttl = int(num_passes), int(init_num_passes)
        self.buffers: List[Any] = [None] * self.size
        self.ttl = [0] * self.size
        self.idx = 0

    def get(self):
        if self.ttl[self.idx] <= 0:
            self.buffers[self.idx] = self.inqueue.get(timeout=self.timeout)
            self.ttl[self.idx] = self.cur_max_ttl
            if self.cur_max_ttl < self.max_ttl:
                self.cur_max_ttl += 1
        buf = self.buffers[self.idx]
        self.ttl[self.idx] -= 1
        released = self.ttl[self.idx] <= 0
        if released:
            self.buffers[self.idx] = None
        self.idx = (self.idx + 1) % self.size
        return buf, released


class LearnerThread(threading.Thread):
    """Background learner: takes batches from ``inqueue``, runs ``learn_fn(batch)`` (a policy's
    ``learn_on_batch`` or ``train_one_step`` bound to an algorithm) ``num_sgd_iter`` times via a
    MinibatchBuffer, and puts ``(env_steps, results)`` on ``outqueue``."""

    def __init__(self, local_worker=None, minibatch_buffer_size: int = 1, num_sgd_iter: int = 1,
                 learner_queue_size: int = 16, learner_queue_timeout: float = 300, *, learn_fn=None):
        super().__init__(daemon=True)
        self.local_worker = local_worker
        self.learn_fn = learn_fn or getattr(local_worker, "learn_on_batch", None)
        if self.learn_fn is None:
            raise ValueError("LearnerThread needs learn_fn or a local_worker with learn_on_batch")
        self.inqueue: "queue.Queue" = queue.Queue(maxsize=learner_queue_size)
        self.outqueue: "queue.Queue" = queue.Queue()
        self.minibatch_buffer = MinibatchBuffer(self.inqueue, minibatch_buffer_size, learner_queue_timeout,
                                                num_sgd_iter)
        self.stopped = False
        self.learner_info: Dict = {}
        self.num_steps = 0

    def run(self):
        while not self.stopped:
            self.step()

    def step(self):
        try:
            batch, _ = self.minibatch_buffer.get()
        except queue.Empty:
            return
        t0 = time.perf_counter()
        self.learner_info = self.learn_fn(batch) or {}
        self.learner_info.setdefault("learn_time_ms", 1e3 * (time.perf_counter() - t0))
        self.num_steps += 1
        self.outqueue.put((len(batch), self.learner_info))

    def stop(self):
        self.stopped = True


class MultiGPULearnerThread(LearnerThread):
    """Same loop; the learn function is expected to spread the batch over several GPUs (the
    LearnerGroup does, over RCCL)."""

    def __init__(self, local_worker=None, num_gpus: int = 1, **kw):
        super().__init__(local_worker, **kw)
        self.num_gpus = num_gpus


__all__ = ["multi_gpu_train_one_step", "standardize_fields", "synchronous_parallel_sample", "train_one_step",
           "LearnerThread", "MultiGPULearnerThread", "SimpleReplayBuffer", "MinibatchBuffer"]
