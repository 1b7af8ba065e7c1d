"""Trial schedulers (reference: ``python/ray/tune/schedulers``): FIFO, ASHA, HyperBand (async
successive-halving brackets), MedianStoppingRule, PopulationBasedTraining."""
from __future__ import annotations

import copy
import math
import random
from collections import defaultdict
from typing import Callable, Dict, List, Optional

import numpy as np


class TrialScheduler:
    CONTINUE = "CONTINUE"
    PAUSE = "PAUSE"
    STOP = "STOP"
    NOOP = "NOOP"

    def __init__(self, metric=None, mode=None):
        self.metric = metric
        self.mode = mode

    def set_search_properties(self, metric, mode, **spec):
        if self.metric is None:
            self.metric = metric
        if self.mode is None:
            self.mode = mode
        return True

    def _score(self, result):
        v = result.get(self.metric)
        if v is None:
            return None
        return float(v) if self.mode != "min" else -float(v)

    def on_trial_add(self, controller, trial):
        pass

    def on_trial_result(self, controller, trial, result) -> str:
        return TrialScheduler.CONTINUE

    def on_trial_complete(self, controller, trial, result):
        pass

    def on_trial_error(self, controller, trial):
        pass

    def on_trial_remove(self, controller, trial):
        pass

    def choose_trial_to_run(self, controller):
        return None


class FIFOScheduler(TrialScheduler):
    pass


class AsyncHyperBandScheduler(TrialScheduler):
    """ASHA: asynchronous successive halving over rungs at grace_period * rf^k."""

    def __init__(self, time_attr: str = "training_iteration", metric=None, mode=None, max_t: float = 100,
                 grace_period: float = 1, reduction_factor: float = 4, brackets: int = 1,
                 stop_last_trials: bool = True):
        super().__init__(metric, mode)
        if grace_period <= 0 or reduction_factor <= 1 or max_t <= 0:
            raise ValueError("invalid ASHA parameters")
        self.time_attr = time_attr
        self.max_t = max_t
        self.rf = reduction_factor
        self.brackets = []
        for s in range(brackets):
            rungs = []
            t = grace_period * (reduction_factor ** s)
            while t < max_t:
                rungs.append(t)
                t *= reduction_factor
            self.brackets.append({"rungs": rungs, "recorded": defaultdict(list)})
        self._trial_bracket = {}
        self._next = 0

    def on_trial_add(self, controller, trial):
        self._trial_bracket[trial.trial_id] = self._next % len(self.brackets)
        self._next += 1

    def on_trial_result(self, controller, trial, result):
        t = result.get(self.time_attr)
        if t is None:
            return self.CONTINUE
        if t >= self.max_t:
            return self.STOP
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        b = self.brackets[self._trial_bracket.get(trial.trial_id, 0)]
        action = self.CONTINUE
        for milestone in reversed(b["rungs"]):
            if t < milestone:
                continue
            rec = b["recorded"][milestone]
            if trial.trial_id in [r[0] for r in rec]:
                break
            rec.append((trial.trial_id, s))
            scores = [x[1] for x in rec]
            if len(scores) > 1:
                cutoff = np.nanpercentile(scores, (1 - 1 / self.rf) * 100)
                if s < cutoff:
                    action = self.STOP
            break
        return action


ASHAScheduler = AsyncHyperBandScheduler


class HyperBandScheduler(AsyncHyperBandScheduler):
    """HyperBand as multiple asynchronous successive-halving brackets (no synchronous pausing)."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None, max_t=81, reduction_factor=3,
                 stop_last_trials=True):
        nb = max(1, int(math.log(max_t) / math.log(reduction_factor)) + 1)
        super().__init__(time_attr, metric, mode, max_t, 1, reduction_factor, brackets=nb)


class MedianStoppingRule(TrialScheduler):
    def __init__(self, time_attr="time_total_s", metric=None, mode=None, grace_period=60.0, min_samples_required=3,
                 min_time_slice=0, hard_stop=True):
        super().__init__(metric, mode)
        self.time_attr = time_attr
        self.grace = grace_period
        self.min_samples = min_samples_required
        self.hard_stop = hard_stop
        self.hist: Dict[str, List[tuple]] = defaultdict(list)
        self.completed = set()

    def on_trial_result(self, controller, trial, result):
        t = result.get(self.time_attr, 0)
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        self.hist[trial.trial_id].append((t, s))
        if t < self.grace:
            return self.CONTINUE
        others = []
        for tid, h in self.hist.items():
            if tid == trial.trial_id:
                continue
            upto = [x[1] for x in h if x[0] <= t]
            if upto:
                others.append(np.mean(upto))
        if len(others) < self.min_samples:
            return self.CONTINUE
        best = max(x[1] for x in self.hist[trial.trial_id])
        if best < np.median(others):
            return self.STOP if self.hard_stop else self.PAUSE
        return self.CONTINUE


class PopulationBasedTraining(TrialScheduler):
    """PBT: every ``perturbation_interval`` the bottom quantile clones a top-quantile trial's
    checkpoint and a perturbed config (controller restarts the trial from that checkpoint)."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None, perturbation_interval=60.0,
                 burn_in_period=0.0, hyperparam_mutations=None, quantile_fraction=0.25, resample_probability=0.25,
                 perturbation_factors=(1.2, 0.8), custom_explore_fn=None, log_config=True, synch=False,
                 require_attrs=True, seed=None):
        super().__init__(metric, mode)
        if not hyperparam_mutations and not custom_explore_fn:
            raise ValueError("You must specify at least one of `hyperparam_mutations` or `custom_explore_fn`")
        self.time_attr = time_attr
        self.interval = perturbation_interval
        self.burn_in = burn_in_period
        self.mutations = hyperparam_mutations or {}
        self.q = quantile_fraction
        self.resample_p = resample_probability
        self.factors = perturbation_factors
        self.custom_explore_fn = custom_explore_fn
        self.last_perturb: Dict[str, float] = {}
        self.scores: Dict[str, float] = {}
        self.num_perturbations = 0
        self._rng = random.Random(seed)

    def _explore(self, config):
        from .. import search as S
        from ..search.sample import Domain

        new = copy.deepcopy(config)
        for k, spec in self.mutations.items():
            if isinstance(spec, dict) and not isinstance(spec, Domain):
                new[k] = self._explore_nested(new.get(k, {}), spec)
                continue
            if self._rng.random() < self.resample_p or k not in new:
                new[k] = spec.sample() if isinstance(spec, Domain) else (
                    self._rng.choice(spec) if isinstance(spec, list) else spec())
            elif isinstance(spec, list):
                i = spec.index(new[k]) if new[k] in spec else 0
                i = max(0, min(len(spec) - 1, i + self._rng.choice([-1, 1])))
                new[k] = spec[i]
            else:
                v = new[k] * self._rng.choice(list(self.factors))
                new[k] = type(new[k])(v) if isinstance(new[k], int) else v
        if self.custom_explore_fn:
            new = self.custom_explore_fn(new)
        return new

    def _explore_nested(self, sub, spec):
        saved = self.mutations
        self.mutations = spec
        try:
            return self._explore(sub)
        finally:
            self.mutations = saved

    def on_trial_result(self, controller, trial, result):
        t = result.get(self.time_attr)
        s = self._score(result)
        if t is None or s is None:
            return self.CONTINUE
        self.scores[trial.trial_id] = s
        if t < self.burn_in:
            return self.CONTINUE
        last = self.last_perturb.get(trial.trial_id, 0)
        if t - last < self.interval:
            return self.CONTINUE
        self.last_perturb[trial.trial_id] = t
        ranked = sorted(self.scores.items(), key=lambda kv: kv[1])
        n = len(ranked)
        k = max(1, int(math.ceil(n * self.q))) if n > 1 else 0
        if k == 0 or n < 2:
            return self.CONTINUE
        bottom = {tid for tid, _ in ranked[:k]}
        top = [tid for tid, _ in ranked[-k:]]
        if trial.trial_id in bottom and trial.trial_id not in top:
            donor_id = self._rng.choice(top)
            donor = controller.get_trial(donor_id)
            if donor is not None and donor.checkpoint is not None:
                new_cfg = self._explore(donor.config)
                self.num_perturbations += 1
                controller.exploit(trial, donor, new_cfg)
                return self.NOOP
        return self.CONTINUE


class PopulationBasedTrainingReplay(TrialScheduler):  # pragma: no cover
    pass


class HyperBandForBOHB(HyperBandScheduler):
    """HyperBand variant paired with a BOHB searcher in the reference (``hb_bohb.py``); the
    successive-halving rungs are the same as HyperBand's here."""


class ResourceChangingScheduler(TrialScheduler):
    """Wraps a base scheduler and, on each result, asks ``resources_allocation_function(controller,
    trial, result, scheduler)`` for new trial resources (reference ``resource_changing_scheduler.py``).
    The new request is recorded on the trial (``trial.resources``) and applies from its next start."""

    def __init__(self, base_scheduler: Optional[TrialScheduler] = None, resources_allocation_function=None):
        super().__init__()
        self.base = base_scheduler or FIFOScheduler()
        self.fn = resources_allocation_function
        self.changes: List[tuple] = []

    def set_search_properties(self, metric, mode, **spec):
        self.metric, self.mode = metric, mode
        return self.base.set_search_properties(metric, mode, **spec)

    def on_trial_add(self, controller, trial):
        return self.base.on_trial_add(controller, trial)

    def on_trial_result(self, controller, trial, result):
        if self.fn is not None:
            new = self.fn(controller, trial, result, self)
            if new is not None:
                res = getattr(new, "required_resources", new)
                if dict(res) != dict(getattr(trial, "resources", {}) or {}):
                    trial.resources = dict(res)
                    self.changes.append((getattr(trial, "trial_id", None), dict(res)))
        return self.base.on_trial_result(controller, trial, result)

    def on_trial_complete(self, controller, trial, result):
        return self.base.on_trial_complete(controller, trial, result)

    def on_trial_error(self, controller, trial):
        return self.base.on_trial_error(controller, trial)

    def choose_trial_to_run(self, controller):
        return self.base.choose_trial_to_run(controller)


__all__ = ["HyperBandForBOHB", "ResourceChangingScheduler", "TrialScheduler", "FIFOScheduler", "AsyncHyperBandScheduler", "ASHAScheduler", "HyperBandScheduler",
           "MedianStoppingRule", "PopulationBasedTraining"]


def __getattr__(name):
    if name == "PB2":
        from .pb2 import PB2

        return PB2
    raise AttributeError(name)
