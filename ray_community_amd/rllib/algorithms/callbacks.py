"""User hooks into the RL training loop (reference: ``rllib/algorithms/callbacks.py``
``DefaultCallbacks`` / ``RLlibCallback`` and ``make_multi_callbacks``).

Set with ``config.callbacks(MyCallbacks)``. Algorithm-side hooks run in the driver
(``on_algorithm_init``, ``on_train_result``, ``on_evaluate_start/end``, ``on_checkpoint_loaded``);
runner-side hooks run inside every env runner actor (``on_environment_created``,
``on_episode_start/step/end``, ``on_sample_end``). Env runners step N sub-envs as one vectorised
batch, so episode hooks receive the sub-env index and an :class:`Episode` record per sub-env;
``on_episode_step`` is only dispatched when a subclass overrides it (per-step Python calls for
every sub-env are otherwise skipped). Values put into ``episode.custom_metrics`` are aggregated into
the train result as ``custom_metrics/<key>_{mean,min,max}`` (reference old-stack behaviour).
"""
from __future__ import annotations

import itertools
from typing import Any, Dict, List, Optional, Type

_EP_IDS = itertools.count()


class Episode:
    """One sub-env episode as seen by the callbacks."""

    __slots__ = ("episode_id", "env_index", "total_reward", "length", "custom_metrics", "user_data", "hist_data",
                 "last_info")

    def __init__(self, env_index: int):
        self.episode_id = next(_EP_IDS)
        self.env_index = env_index
        self.total_reward = 0.0
        self.length = 0
        self.custom_metrics: Dict[str, float] = {}
        self.user_data: Dict[str, Any] = {}
        self.hist_data: Dict[str, List[float]] = {}
        self.last_info: Any = None

    # new-stack spellings
    def get_return(self) -> float:
        return self.total_reward

    def __len__(self):
        return self.length


class DefaultCallbacks:
    """Base class: every hook is a no-op; override the ones you need (keyword arguments only)."""

    # ---------------------------------------------------------------- algorithm side
    def on_algorithm_init(self, *, algorithm, **kwargs) -> None:
        pass

    def on_train_result(self, *, algorithm, result: dict, **kwargs) -> None:
        pass

    def on_evaluate_start(self, *, algorithm, **kwargs) -> None:
        pass

    def on_evaluate_end(self, *, algorithm, evaluation_metrics: dict, **kwargs) -> None:
        pass

    def on_checkpoint_loaded(self, *, algorithm, **kwargs) -> None:
        pass

    def on_workers_recreated(self, *, algorithm, worker_set=None, worker_ids=None, is_evaluation=False,
                             **kwargs) -> None:
        pass

    # ---------------------------------------------------------------- env runner side
    def on_environment_created(self, *, env_runner, env, env_context=None, **kwargs) -> None:
        pass

    def on_episode_start(self, *, episode: Episode, env_runner=None, env_index: int = 0, **kwargs) -> None:
        pass

    def on_episode_step(self, *, episode: Episode, env_runner=None, env_index: int = 0, **kwargs) -> None:
        pass

    def on_episode_end(self, *, episode: Episode, env_runner=None, env_index: int = 0, **kwargs) -> None:
        pass

    def on_sample_end(self, *, env_runner=None, samples=None, **kwargs) -> None:
        pass

    def on_create_policy(self, *, policy_id, policy, **kwargs) -> None:
        """A policy was created (add_policy / multi-agent setup)."""

    def on_episode_created(self, *, episode, env_runner=None, env_index: int = 0, env=None, **kwargs) -> None:
        """A new episode object exists, before its first reset observation."""

    def on_postprocess_trajectory(self, *, episode=None, agent_id=None, policy_id=None, policies=None,
                                  postprocessed_batch=None, original_batches=None, **kwargs) -> None:
        """A trajectory's batch was post-processed (advantages etc.); may edit it in place."""

    def on_sub_environment_created(self, *, worker=None, sub_environment=None, env_context=None, env_index=None,
                                   **kwargs) -> None:
        """One sub-environment of a vectorised env was created."""

    def on_learn_on_batch(self, *, policy=None, train_batch=None, result=None, **kwargs) -> None:
        pass


RLlibCallback = DefaultCallbacks


def overrides(cb: Optional[DefaultCallbacks], name: str) -> bool:
    """True if ``cb`` implements hook ``name`` itself (not the base no-op)."""
    if cb is None:
        return False
    if isinstance(cb, _MultiCallbacks):
        return any(overrides(c, name) for c in cb._cbs)
    return getattr(type(cb), name, None) is not getattr(DefaultCallbacks, name)


class _MultiCallbacks(DefaultCallbacks):
    _classes: List[Type[DefaultCallbacks]] = []

    def __init__(self):
        self._cbs = [c() for c in self._classes]

    def __getattribute__(self, name):
        if name.startswith("on_"):
            cbs = object.__getattribute__(self, "_cbs")

            def fan_out(**kw):
                for c in cbs:
                    getattr(c, name)(**kw)

            return fan_out
        return object.__getattribute__(self, name)


def make_multi_callbacks(callback_class_list: List[Type[DefaultCallbacks]]) -> Type[DefaultCallbacks]:
    """One callbacks class that calls each of ``callback_class_list`` in order."""
    return type("MultiCallbacks", (_MultiCallbacks,), {"_classes": list(callback_class_list)})


def build(cls_or_obj) -> Optional[DefaultCallbacks]:
    if cls_or_obj is None:
        return None
    if isinstance(cls_or_obj, DefaultCallbacks):
        return cls_or_obj
    if isinstance(cls_or_obj, (list, tuple)):
        return make_multi_callbacks(list(cls_or_obj))()
    return cls_or_obj()


def aggregate_custom_metrics(rows: List[Dict[str, float]]) -> Dict[str, float]:
    out: Dict[str, List[float]] = {}
    for r in rows:
        for k, v in r.items():
            out.setdefault(k, []).append(float(v))
    res = {}
    for k, vs in out.items():
        res[f"{k}_mean"] = sum(vs) / len(vs)
        res[f"{k}_min"] = min(vs)
        res[f"{k}_max"] = max(vs)
    return res


__all__ = ["DefaultCallbacks", "RLlibCallback", "Episode", "make_multi_callbacks"]
