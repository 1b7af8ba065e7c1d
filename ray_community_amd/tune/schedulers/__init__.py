"""Trial schedulers (reference: ``python/ray/tune/schedulers``): FIFO, ASHA (asynchronous
successive halving), synchronous HyperBand (+ the BOHB variant), MedianStoppingRule,
PopulationBasedTraining (+ replay of its policy log), ResourceChangingScheduler."""
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

    supports_buffered_results = True

    def debug_string(self) -> str:
        return f"Using {type(self).__name__} (metric={self.metric!r}, mode={self.mode!r})."

    def save(self, checkpoint_path: str) -> None:
        import pickle

        import cloudpickle

        state = {}
        for k, v in self.__dict__.items():
            try:
                cloudpickle.dumps(v)
            except Exception:
                continue
            state[k] = v
        with open(checkpoint_path, "wb") as f:
            cloudpickle.dump(state, f)

    def restore(self, checkpoint_path: str) -> None:
        import pickle

        with open(checkpoint_path, "rb") as f:  # a file this framework's save() wrote
            self.__dict__.update(pickle.load(f))

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


class HyperBandScheduler(TrialScheduler):
    """Synchronous HyperBand (Li et al. 2017; reference ``python/ray/tune/schedulers/hyperband.py``).

    Trials are dealt into brackets s = s_max .. 0 (s_max = floor(log_eta(max_t))); bracket s
    takes n_s = ceil((s_max + 1) / (s + 1) * eta^s) trials starting at budget r_s = max_t * eta^-s.
    Each bracket runs successive halving SYNCHRONOUSLY: a trial that reaches the bracket's current
    milestone is PAUSED (checkpointed, actor released); once every live trial of the (filled)
    bracket has reached it, the top 1/eta continue to milestone * eta and the rest are stopped.
    A bracket counts as filled when it holds n_s trials or the searcher has no more trials.
    """

    manages_paused_trials = True

    def __init__(self, time_attr="training_iteration", metric=None, mode=None, max_t=81, reduction_factor=3,
                 stop_last_trials=True):
        super().__init__(metric, mode)
        if max_t <= 0 or reduction_factor <= 1:
            raise ValueError("invalid HyperBand parameters")
        self.time_attr = time_attr
        self.max_t = max_t
        self.eta = reduction_factor
        self.stop_last_trials = stop_last_trials
        self.s_max = int(math.floor(math.log(max_t) / math.log(reduction_factor) + 1e-9))
        self.brackets: List[Dict] = []
        self._trial_bracket: Dict[str, Dict] = {}
        self._next_s = self.s_max
        self.decisions: List[tuple] = []  # (bracket index, milestone, kept ids, stopped ids)

    def state(self) -> Dict:
        """Bracket bookkeeping: per bracket its budget, size, trial ids and current milestone."""
        return {"num_brackets": len(self.brackets), "s_max": self.s_max,
                "brackets": [{k: (sorted(v) if isinstance(v, set) else v) for k, v in b.items()
                              if isinstance(v, (int, float, str, list, set))} for b in self.brackets]}

    def _new_bracket(self):
        s = self._next_s
        self._next_s = self._next_s - 1 if self._next_s > 0 else self.s_max
        n = int(math.ceil((self.s_max + 1) / (s + 1) * self.eta ** s))
        r = self.max_t * self.eta ** (-s)
        b = {"index": len(self.brackets), "s": s, "n": n, "milestone": max(1.0, r), "trials": [], "live": set(),
             "reached": {}}
        self.brackets.append(b)
        return b

    def on_trial_add(self, controller, trial):
        b = self.brackets[-1] if self.brackets and len(self.brackets[-1]["trials"]) < self.brackets[-1]["n"] else \
            self._new_bracket()
        b["trials"].append(trial.trial_id)
        b["live"].add(trial.trial_id)
        self._trial_bracket[trial.trial_id] = b

    def _filled(self, controller, b) -> bool:
        return len(b["trials"]) >= b["n"] or getattr(controller, "searcher_done", False)

    def on_trial_result(self, controller, trial, result):
        t = result.get(self.time_attr)
        b = self._trial_bracket.get(trial.trial_id)
        if t is None or b is None:
            return self.CONTINUE
        if t >= self.max_t:
            b["live"].discard(trial.trial_id)
            return self.STOP if self.stop_last_trials else self.CONTINUE
        if t < b["milestone"]:
            return self.CONTINUE
        s = self._score(result)
        b["reached"][trial.trial_id] = -math.inf if s is None else s
        decision = self._maybe_halve(controller, b, current=trial.trial_id)
        return decision if decision is not None else self.PAUSE

    def on_trial_complete(self, controller, trial, result):
        b = self._trial_bracket.get(trial.trial_id)
        if b is not None:
            b["live"].discard(trial.trial_id)
            b["reached"].pop(trial.trial_id, None)
            self._maybe_halve(controller, b)

    def on_trial_error(self, controller, trial):
        self.on_trial_complete(controller, trial, None)

    def _maybe_halve(self, controller, b, current=None):
        """Run successive halving on bracket ``b`` if every live trial reached its milestone.
        Returns the decision for ``current`` (the trial whose result triggered it), if any."""
        if not b["live"] or not self._filled(controller, b) or not set(b["live"]) <= set(b["reached"]):
            return None
        ranked = sorted(b["live"], key=lambda tid: b["reached"][tid], reverse=True)
        k = max(1, int(len(ranked) // self.eta))
        keep, cut = ranked[:k], ranked[k:]
        self.decisions.append((b["index"], b["milestone"], list(keep), list(cut)))
        b["milestone"] = min(self.max_t, b["milestone"] * self.eta)
        b["reached"] = {}
        b["live"] = set(keep)
        out = None
        for tid in keep:
            if tid == current:
                out = self.CONTINUE
            else:
                tr = controller.get_trial(tid)
                if tr is not None:
                    controller.unpause(tr)
        for tid in cut:
            if tid == current:
                out = self.STOP
            else:
                tr = controller.get_trial(tid)
                if tr is not None:
                    controller.stop_paused(tr)
        return out

    def choose_trial_to_run(self, controller):
        # the searcher ran dry: brackets that will never fill are halved with what they have
        if getattr(controller, "searcher_done", False):
            for b in self.brackets:
                self._maybe_halve(controller, b)
        return None


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
        self.log_config = log_config
        self.scores: Dict[str, float] = {}
        self.num_perturbations = 0
        self._rng = random.Random(seed)

    def reset_stats(self) -> None:
        """Forget the recorded scores and perturbation times (e.g. between experiments)."""
        self.scores = {}
        self.last_perturb = {}
        self.num_perturbations = 0

    def last_scores(self, trials) -> List[float]:
        """The latest recorded score of each trial that has one (higher is better)."""
        return [self.scores[t.trial_id] for t in trials if t.trial_id in self.scores]

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

    def _log_policy(self, controller, trial, donor, new_cfg):
        """One JSON line per exploit in ``pbt_policy_<trial_id>.txt`` (what
        PopulationBasedTrainingReplay reads back)."""
        import json
        import os

        d = getattr(controller, "exp_dir", None)
        if not d or not self.log_config:
            return
        row = [donor.trial_id, trial.trial_id, donor.last_result.get(self.time_attr, 0),
               trial.last_result.get(self.time_attr, 0), donor.config, new_cfg]
        try:
            with open(os.path.join(d, f"pbt_policy_{trial.trial_id}.txt"), "a") as f:
                f.write(json.dumps(row, default=str) + "\n")
        except OSError:
            pass

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
                self._log_policy(controller, trial, donor, new_cfg)
                controller.exploit(trial, donor, new_cfg)
                return self.NOOP
        return self.CONTINUE


class PopulationBasedTrainingReplay(TrialScheduler):
    """Replays the hyperparameter schedule one trial followed in a PBT run (reference
    ``pbt.py`` ``PopulationBasedTrainingReplay``): the policy log PBT writes for every exploit
    (``pbt_policy_<trial_id>.txt`` in the experiment directory, one JSON line per change:
    ``[old_trial, new_trial, old_step, new_step, old_config, new_config]``) becomes a list of
    (step, config) changes. The replayed trial starts from the first logged config and, when its
    ``time_attr`` reaches a change point, is checkpointed and restarted with that config."""

    def __init__(self, policy_file: str, time_attr: str = "training_iteration"):
        super().__init__()
        import json

        self.time_attr = time_attr
        with open(policy_file) as f:
            rows = [json.loads(l) for l in f if l.strip()]
        if not rows:
            raise ValueError(f"policy file {policy_file} holds no PBT changes")
        self.config = dict(rows[0][4])
        self._changes = [(int(r[3]), dict(r[5])) for r in rows]
        self._i = 0
        self.applied: List[tuple] = []

    def on_trial_add(self, controller, trial):
        trial.config = dict(self.config)

    def on_trial_result(self, controller, trial, result):
        t = result.get(self.time_attr)
        if t is None or self._i >= len(self._changes):
            return self.CONTINUE
        step, cfg = self._changes[self._i]
        if t < step:
            return self.CONTINUE
        self._i += 1
        self.applied.append((t, cfg))
        controller.restart(trial, new_config=cfg)
        return self.NOOP


class HyperBandForBOHB(HyperBandScheduler):
    """Synchronous HyperBand paired with the ``TuneBOHB`` searcher (reference ``hb_bohb.py``): the
    searcher sees every milestone result with its budget (``time_attr``), so its model is fitted
    on the largest budget that has enough observations."""


class ResourceChangingScheduler(TrialScheduler):
    """Wraps a base scheduler; on each result ``resources_allocation_function(controller, trial,
    result, scheduler)`` may return new trial resources (a dict or a ``PlacementGroupFactory``;
    reference ``resource_changing_scheduler.py``). A change checkpoints the trial and restarts it
    from that checkpoint in a trial actor of the new size."""

    def __init__(self, base_scheduler: Optional[TrialScheduler] = None, resources_allocation_function=None):
        super().__init__()
        self.base = base_scheduler or FIFOScheduler()
        self.fn = resources_allocation_function
        self.changes: List[tuple] = []

    @property
    def manages_paused_trials(self):
        return getattr(self.base, "manages_paused_trials", False)

    def set_search_properties(self, metric, mode, **spec):
        self.metric, self.mode = metric, mode
        return self.base.set_search_properties(metric, mode, **spec)

    def on_trial_add(self, controller, trial):
        return self.base.on_trial_add(controller, trial)

    def on_trial_result(self, controller, trial, result):
        decision = self.base.on_trial_result(controller, trial, result)
        if decision != self.CONTINUE or self.fn is None:
            return decision
        new = self.fn(controller, trial, result, self)
        if new is None:
            return decision
        res = getattr(new, "required_resources", new)
        res = {k: v for k, v in dict(res).items() if v}
        if res != {k: v for k, v in dict(getattr(trial, "resources", {}) or {}).items() if v}:
            self.changes.append((getattr(trial, "trial_id", None), dict(res)))
            controller.restart(trial, new_resources=res)
            return self.NOOP
        return decision

    def on_trial_complete(self, controller, trial, result):
        return self.base.on_trial_complete(controller, trial, result)

    def on_trial_error(self, controller, trial):
        return self.base.on_trial_error(controller, trial)

    def choose_trial_to_run(self, controller):
        return self.base.choose_trial_to_run(controller)


__all__ = ["HyperBandForBOHB", "ResourceChangingScheduler", "PopulationBasedTrainingReplay", "TrialScheduler", "FIFOScheduler", "AsyncHyperBandScheduler", "ASHAScheduler", "HyperBandScheduler",
           "MedianStoppingRule", "PopulationBasedTraining"]


def __getattr__(name):
    if name == "PB2":
        from .pb2 import PB2

        return PB2
    raise AttributeError(name)
