"""IMPALA and APPO (reference: ``rllib/algorithms/impala/impala.py``, ``vtrace_torch.py``,
``rllib/algorithms/appo/appo.py``).

Asynchronous actor-learner architecture: every env runner keeps
``max_requests_in_flight_per_env_runner`` sample requests queued; each ``training_step`` takes
whichever fragments are ready (``wait``), immediately re-queues those runners, and trains on the
concatenated ``[N, T]`` fragments. Runners therefore act with weights that lag the learner by a
few updates; V-trace (a HIP kernel over the env-major fragments, ``ops.vtrace``) corrects for the
policy lag. Weights are broadcast without blocking every ``broadcast_interval`` updates (actor
calls are ordered per caller, so a runner's next fragment uses them).

Learner queue (reference ``rllib/execution/learner_thread.py``, ``impala.py``
``place_processed_samples_on_learner_thread_queue``): with ``learner_queue_size > 0`` (default 16)
a background learner thread owns the LearnerGroup updates. ``training_step`` only samples and
enqueues train batches (blocking for at most ``learner_queue_timeout`` seconds when the queue is
full) and collects whatever updates finished meanwhile, so sampling continues while the learner
trains; the learner thread snapshots the weights after every ``broadcast_interval`` updates and
the next ``training_step`` broadcasts them. ``learner_queue_size = 0`` trains inline.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Dict, List

from ..policy.sample_batch import concat_samples
from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig


class IMPALAConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or IMPALA)
        self.vtrace = True
        self.vtrace_clip_rho_threshold = 1.0
        self.vtrace_clip_c_threshold = 1.0
        self.vtrace_clip_pg_rho_threshold = 1.0
        self.lr = 0.0005
        self.train_batch_size = 500
        self.rollout_fragment_length = 50
        self.vf_loss_coeff = 0.5
        self.entropy_coeff = 0.01
        self.grad_clip = 40.0
        self.broadcast_interval = 1
        self.max_requests_in_flight_per_env_runner = 2
        self.num_epochs = 1
        self.minibatch_size = None
        self.learner_queue_size = 16
        self.learner_queue_timeout = 300


class IMPALA(Algorithm):
    _default_config_cls = IMPALAConfig
    _update_kind = "impala"

    @classmethod
    def get_default_config(cls):
        return cls._default_config_cls()

    def _sample_async(self, steps: int):
        from ..._private.worker import get, wait

        cfg = self.config
        g = self.env_runner_group
        frag = cfg.get_rollout_fragment_length() * max(1, cfg.num_envs_per_env_runner)
        if not hasattr(self, "_inflight"):
            self._inflight = {}  # sample ref -> runner id
        # top every healthy runner (new, or restored by restore_workers) up to its request budget
        actors = g.manager.actors()
        per = max(1, cfg.max_requests_in_flight_per_env_runner)
        for i in g.healthy_env_runner_ids():
            for _ in range(per - sum(1 for v in self._inflight.values() if v == i)):
                self._inflight[actors[i].sample.remote(frag)] = i
        got: List = []
        n = 0
        while n < steps:
            if not self._inflight:  # no healthy remote runner left: the local one samples
                b = self.local_runner.sample(max(steps - n, self.local_runner.N))
                got.append(b)
                n += b.count
                break
            ready, _ = wait(list(self._inflight), num_returns=1)
            for ref in ready:
                i = self._inflight.pop(ref)
                try:
                    b = get(ref)
                except Exception as e:  # noqa  (the group's policy decides: raise, or drop the runner)
                    g.mark_failed(i, e)
                    for other in [r for r, j in self._inflight.items() if j == i]:
                        self._inflight.pop(other, None)
                    continue
                got.append(b)
                n += b.count
                if g.manager.is_actor_healthy(i):
                    self._inflight[g.manager.actors()[i].sample.remote(frag)] = i
        return concat_samples(got)

    def _broadcast_async(self):
        from ..._private.worker import put

        st = self.learner_group.get_weights()
        self._weights_version += 1
        self.local_runner.set_weights(st, self._weights_version)
        if self.remote_runners:
            ref = put(st)
            for r in self.remote_runners:
                r.set_weights.remote(ref, self._weights_version)

    def training_step(self) -> Dict:
        cfg = self.config
        if int(getattr(cfg, "learner_queue_size", 0) or 0) > 0:
            return self._training_step_queued()
        batch = self._sample_async(cfg.train_batch_size)
        n = batch.count
        self._timesteps_total += n
        info = self.learner_group.update(self._update_kind, batch)
        self._num_updates = getattr(self, "_num_updates", 0) + 1
        if self._num_updates % max(1, cfg.broadcast_interval) == 0:
            self._broadcast_async()
        info["_steps_this_iter"] = n
        info["num_weight_broadcasts"] = self._weights_version
        return info

    # ------------------------------------------------------------------ learner thread
    def _start_learner_thread(self):
        cfg = self.config
        self._lq = queue.Queue(maxsize=int(cfg.learner_queue_size))
        self._lq_out = queue.Queue()
        self._lq_stop = threading.Event()
        self._lq_lock = threading.Lock()  # held around every update (checkpointing takes it too)
        self._lq_weights = None  # (update count, weights) snapshot awaiting broadcast
        self._lq_updates = 0
        self._lq_error = None
        # (start, end) wall times of the learner's updates and of the driver's sample collections:
        # what ``learner_overlap_s`` (sampling while the learner trains) is computed from
        self._lq_update_spans: List = []
        self._sample_spans: List = []
        self._lq_wait_s = 0.0  # driver time blocked on learner results
        self._lq_busy_s = 0.0  # learner-thread update time
        every = max(1, int(cfg.broadcast_interval))

        def run():
            while not self._lq_stop.is_set():
                try:
                    batch = self._lq.get(timeout=0.05)
                except queue.Empty:
                    continue
                try:
                    t0 = time.perf_counter()
                    with self._lq_lock:
                        info = self.learner_group.update(self._update_kind, batch)
                        self._lq_updates += 1
                        if self._lq_updates % every == 0:
                            self._lq_weights = (self._lq_updates, self.learner_group.get_weights())
                    t1 = time.perf_counter()
                    self._lq_busy_s += t1 - t0
                    self._lq_update_spans.append((t0, t1))
                    del self._lq_update_spans[:-256]
                    self._lq_out.put(info)
                except BaseException as e:  # noqa: BLE001 -- surfaced by the next training_step
                    self._lq_error = e
                    return

        self._lq_thread = threading.Thread(target=run, name="rllib-learner-thread", daemon=True)
        self._lq_thread.start()

    def _training_step_queued(self) -> Dict:
        cfg = self.config
        if getattr(self, "_lq_thread", None) is None:
            self._start_learner_thread()
        if self._lq_error is not None:
            raise self._lq_error
        if not self._lq_thread.is_alive():
            raise RuntimeError("The IMPALA learner thread has died")
        t0 = time.perf_counter()
        batch = self._sample_async(cfg.train_batch_size)
        self._sample_spans.append((t0, time.perf_counter()))
        del self._sample_spans[:-256]
        n = batch.count
        self._timesteps_total += n
        try:
            self._lq.put(batch, block=True, timeout=float(cfg.learner_queue_timeout))
        except queue.Full:
            raise RuntimeError(f"the learner queue stayed full for learner_queue_timeout="
                               f"{cfg.learner_queue_timeout} s: the learner is not keeping up") from None
        infos = []
        # the first iteration waits for one result (there is nothing to report otherwise)
        if getattr(self, "_lq_last_info", None) is None:
            infos.append(self._wait_learner_result(float(cfg.learner_queue_timeout)))
        while True:
            try:
                infos.append(self._lq_out.get_nowait())
            except queue.Empty:
                break
        if infos:
            self._lq_last_info = infos[-1]
        snap, self._lq_weights = self._lq_weights, None
        if snap is not None:
            self._broadcast_weights(snap[1])
        self._num_updates = self._lq_updates
        info = dict(self._lq_last_info)
        info["_steps_this_iter"] = n
        info["num_weight_broadcasts"] = self._weights_version
        info["learner_queue_size"] = self._lq.qsize()
        info["num_learner_updates"] = self._lq_updates
        info["num_updates_this_iter"] = len(infos)
        info["learner_overlap_s"] = self._learner_overlap_s()
        return info

    def _wait_learner_result(self, timeout: float):
        t0 = time.perf_counter()
        deadline = time.monotonic() + timeout
        try:
            while True:
                if self._lq_error is not None:
                    raise self._lq_error
                try:
                    return self._lq_out.get(timeout=0.05)
                except queue.Empty:
                    if time.monotonic() > deadline:
                        raise RuntimeError("no learner result within learner_queue_timeout") from None
        finally:
            self._lq_wait_s += time.perf_counter() - t0

    def _learner_overlap_s(self) -> float:
        """Learner-thread update seconds during which the driver was NOT blocked on the learner
        (it was collecting fragments, broadcasting weights or between iterations, while the env
        runners kept sampling): total update time minus the driver's waits for learner results.
        0 means the learner ran inline in effect; > 0 means sampling and learning overlap."""
        return max(0.0, self._lq_busy_s - self._lq_wait_s)

    def _broadcast_weights(self, st):
        from ..._private.worker import put

        self._weights_version += 1
        self.local_runner.set_weights(st, self._weights_version)
        if self.remote_runners:
            ref = put(st)
            for r in self.remote_runners:
                r.set_weights.remote(ref, self._weights_version)

    def _stop_learner_thread(self):
        th = getattr(self, "_lq_thread", None)
        if th is not None:
            self._lq_stop.set()
            th.join(timeout=30)
            self._lq_thread = None

    def save_checkpoint(self, checkpoint_dir: str):
        lock = getattr(self, "_lq_lock", None)
        if lock is None:
            return super().save_checkpoint(checkpoint_dir)
        with lock:  # no update half-applied in the saved learner state
            return super().save_checkpoint(checkpoint_dir)

    def stop(self):
        self._stop_learner_thread()
        self._inflight = {}
        super().stop()

    cleanup = stop


class APPOConfig(IMPALAConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or APPO)
        self.clip_param = 0.4
        self.use_kl_loss = False
        self.kl_coeff = 1.0
        self.kl_target = 0.01
        self.num_epochs = 1
        self.lr = 0.0005
        # target network (reference appo.py): Polyak coefficient and refresh period in learner updates
        self.tau = 1.0
        self.target_update_frequency = 1


class APPO(IMPALA):
    _default_config_cls = APPOConfig
    _update_kind = "appo"
