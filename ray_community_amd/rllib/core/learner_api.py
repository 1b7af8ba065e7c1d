"""The reference's Learner / LearnerGroup / RLModule extension API (rllib/core/learner/learner.py,
learner_group.py, rl_module/rl_module.py) over this framework's learners.

The built-in algorithms train through fused, device-resident updates (``Learner.update_ppo``,
``update_dqn``, ...). Custom learners plug in the reference way: subclass ``Learner`` and override
``compute_loss_for_module(module_id=, config=, batch=, fwd_out=)`` (and optionally
``configure_optimizers_for_module`` / ``postprocess_gradients_for_module``); then
``update_from_batch(batch, minibatch_size=, num_iters=)`` runs the generic loop:
``forward_train`` -> ``compute_loss`` -> ``compute_gradients`` -> ``postprocess_gradients`` ->
``apply_gradients``, with the batch resident on the learner's device and minibatches drawn by a
device-side permutation. Without an override it runs the algorithm's own fused update."""
from __future__ import annotations

import os
import threading
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch

DEFAULT_MODULE_ID = "default_policy"
POLICY_LOSS_KEY, VF_LOSS_KEY, ENTROPY_KEY = "policy_loss", "vf_loss", "entropy"
ALL_MODULES = "__all_modules__"


# ============================================================================ RLModule
class RLModuleAPI:
    """Mixed into RLModule / MultiRLModule (torch ``nn.Module``s with ``forward`` returning
    (logits, value) and ``get_state`` / ``set_state``)."""

    framework = "torch"

    def setup(self) -> None:
        """Hook for subclasses that build layers lazily (the constructor already built them)."""

    def get_initial_state(self, *args, **kwargs) -> Dict:
        return {}

    # a bool attribute here (the runners test ``module.is_stateful``) that is also callable like
    # the reference's ``is_stateful()`` method; RecurrentRLModule sets it to StatefulFlag(1)
    is_stateful = None  # replaced below

    def update_default_view_requirements(self, defaults: Dict) -> Dict:
        return defaults

    def forward_train(self, batch: Dict) -> Dict[str, torch.Tensor]:
        logits, v = self.forward(batch["obs"])
        return {"action_dist_inputs": logits, "vf_preds": v}

    def get_train_action_dist_cls(self):
        return self.dist_cls

    get_exploration_action_dist_cls = get_train_action_dist_cls
    get_inference_action_dist_cls = get_train_action_dist_cls

    def input_specs_train(self) -> List[str]:
        return ["obs", "actions"]

    def input_specs_exploration(self) -> List[str]:
        return ["obs"]

    input_specs_inference = input_specs_exploration

    def output_specs_train(self) -> List[str]:
        return ["action_dist_inputs", "vf_preds"]

    def output_specs_exploration(self) -> List[str]:
        return ["actions", "action_logp", "vf_preds", "action_dist_inputs"]

    def output_specs_inference(self) -> List[str]:
        return ["actions", "vf_preds"]

    def save_state(self, dir: str) -> None:  # noqa: A002 (reference name)
        os.makedirs(dir, exist_ok=True)
        torch.save(self.get_state(), os.path.join(dir, "module_state.pt"))

    def load_state(self, dir: str) -> None:  # noqa: A002
        self.set_state(torch.load(os.path.join(dir, "module_state.pt"), weights_only=True))

    def _ctor_args(self):
        return (getattr(self, "obs_space", None), getattr(self, "act_space", None),
                getattr(self, "model_config", None))

    def save_to_checkpoint(self, checkpoint_dir_path: str) -> None:
        """State plus what rebuilds the module: its class and constructor arguments (spaces,
        model config), pickled with cloudpickle next to ``module_state.pt``."""
        import cloudpickle

        self.save_state(checkpoint_dir_path)
        with open(os.path.join(checkpoint_dir_path, "module_spec.pkl"), "wb") as f:
            cloudpickle.dump((type(self), self._ctor_args()), f)

    @classmethod
    def from_checkpoint(cls, checkpoint_dir_path: str):
        import pickle

        with open(os.path.join(checkpoint_dir_path, "module_spec.pkl"), "rb") as f:  # written by save_to_checkpoint
            klass, args = pickle.load(f)
        m = klass(*args)
        m.load_state(checkpoint_dir_path)
        return m

    def as_multi_agent(self):
        from .rl_module import MultiRLModule

        return MultiRLModule({DEFAULT_MODULE_ID: self})

    def unwrapped(self):
        return self


class StatefulFlag(int):
    """``module.is_stateful`` works as a bool attribute and as the reference's method call."""

    def __call__(self) -> bool:
        return bool(self)

    def __repr__(self):
        return repr(bool(self))


RLModuleAPI.is_stateful = StatefulFlag(0)


class MultiRLModuleAPI(RLModuleAPI):
    def get_initial_state(self, *args, **kwargs) -> Dict:
        return {mid: m.get_initial_state() for mid, m in self.items()
                if hasattr(m, "get_initial_state") and getattr(m, "is_stateful", False)}

    @property
    def is_stateful(self) -> StatefulFlag:
        return StatefulFlag(any(bool(getattr(m, "is_stateful", False)) for m in self.values()))

    def _ctor_args(self):
        return (dict(self.items()),)

    def save_to_checkpoint(self, checkpoint_dir_path: str) -> None:
        for mid, m in self.items():
            m.save_to_checkpoint(os.path.join(checkpoint_dir_path, str(mid)))
        with open(os.path.join(checkpoint_dir_path, "module_ids.txt"), "w") as f:
            f.write("\n".join(str(k) for k in self.keys()))

    @classmethod
    def from_checkpoint(cls, checkpoint_dir_path: str):
        from .rl_module import MultiRLModule

        with open(os.path.join(checkpoint_dir_path, "module_ids.txt")) as f:
            ids = [l.strip() for l in f if l.strip()]
        return MultiRLModule({mid: RLModuleAPI.from_checkpoint.__func__(RLModuleAPI,
                                                                          os.path.join(checkpoint_dir_path, mid))
                              for mid in ids})


# ============================================================================ Learner
class LearnerAPI:
    """Mixed into ``Learner`` (which provides ``module``, ``opt``, ``device``, ``cfg``)."""

    # --------------------------------------------------------------------- structure
    def build(self) -> None:
        """Already built by the constructor (module on the device, optimizer, DDP wrapper)."""

    @property
    def distributed(self) -> bool:
        return self.ddp is not None

    @property
    def config(self) -> Dict:
        return self.cfg

    def _modules(self) -> Dict[str, Any]:
        m = self.module
        return dict(m.items()) if hasattr(m, "items") and callable(m.items) else {DEFAULT_MODULE_ID: m}

    def should_module_be_updated(self, module_id, multi_agent_batch=None) -> bool:
        to_train = self.cfg.get("policies_to_train")
        return to_train is None or module_id in to_train

    def add_module(self, *, module_id, module_spec=None, module=None, **kw):
        from .rl_module import MultiRLModule

        if not isinstance(self.module, MultiRLModule):
            self.module = MultiRLModule({DEFAULT_MODULE_ID: self.module})
        new = module if module is not None else module_spec.build()
        self.module.add_module(module_id, new.to(self.device))
        self.register_optimizer(module_id=module_id, optimizer_name="default_optimizer",
                                optimizer=torch.optim.Adam(new.parameters(), lr=self.cfg.get("lr", 5e-5)),
                                params=list(new.parameters()))
        return self.module

    def remove_module(self, module_id, **kw):
        from .rl_module import MultiRLModule

        if not isinstance(self.module, MultiRLModule):
            raise ValueError("remove_module needs a multi-module learner")
        self.module.remove_module(module_id)
        getattr(self, "_optimizers", {}).pop(module_id, None)
        return self.module

    # --------------------------------------------------------------------- optimizers
    def _opt_table(self) -> Dict[str, Dict[str, Any]]:
        if not hasattr(self, "_optimizers"):
            self._optimizers = {}
        return self._optimizers

    def register_optimizer(self, *, module_id=ALL_MODULES, optimizer_name: str = "default_optimizer",
                           optimizer: torch.optim.Optimizer, params=None, lr_or_lr_schedule=None) -> None:
        self._opt_table().setdefault(module_id, {})[optimizer_name] = optimizer

    def configure_optimizers(self) -> None:
        for mid in self._modules():
            self.configure_optimizers_for_module(module_id=mid, config=self.cfg)

    def configure_optimizers_for_module(self, module_id, config=None) -> None:
        mod = self._modules()[module_id]
        self.register_optimizer(module_id=module_id, optimizer=torch.optim.Adam(
            mod.parameters(), lr=(config or self.cfg).get("lr", 5e-5)), params=list(mod.parameters()))

    def get_optimizer(self, module_id=DEFAULT_MODULE_ID, optimizer_name: str = "default_optimizer"):
        tab = self._opt_table()
        if module_id in tab and optimizer_name in tab[module_id]:
            return tab[module_id][optimizer_name]
        return self.opt  # the built-in learner's single optimizer over the whole module

    def get_optimizers_for_module(self, module_id=DEFAULT_MODULE_ID):
        tab = self._opt_table().get(module_id)
        return list(tab.items()) if tab else [("default_optimizer", self.opt)]

    def filter_param_dict_for_optimizer(self, param_dict: Dict, optimizer) -> Dict:
        ids = {id(p) for g in optimizer.param_groups for p in g["params"]}
        return {k: v for k, v in param_dict.items() if id(self.get_param_ref(v)) in ids}

    def get_optimizer_state(self) -> Dict:
        st = {"default_optimizer": self.opt.state_dict()}
        for mid, opts in self._opt_table().items():
            for name, o in opts.items():
                st[f"{mid}/{name}"] = o.state_dict()
        return st

    def set_optimizer_state(self, state: Dict) -> None:
        for key, s in state.items():
            if key == "default_optimizer":
                self.opt.load_state_dict(s)
            else:
                mid, name = key.split("/", 1)
                self._opt_table()[mid][name].load_state_dict(s)

    # --------------------------------------------------------------------- params / state
    def get_param_ref(self, param):
        return param

    def get_parameters(self, module) -> List[torch.nn.Parameter]:
        return list(module.parameters())

    def get_module_state(self, module_ids=None) -> Dict:
        mods = self._modules()
        ids = list(mods) if module_ids is None else list(module_ids)
        if len(mods) == 1 and ids == [DEFAULT_MODULE_ID]:
            return self.module.get_state()
        return {mid: mods[mid].get_state() for mid in ids}

    def set_module_state(self, state: Dict) -> None:
        mods = self._modules()
        if len(mods) == 1 and not set(state) <= set(mods):
            self.module.set_state(state)
        else:
            for mid, s in state.items():
                mods[mid].set_state(s)

    def save_state(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        torch.save(self.get_state(), os.path.join(path, "learner_state.pt"))

    def load_state(self, path: str) -> None:
        self.set_state(torch.load(os.path.join(path, "learner_state.pt"), weights_only=True))

    # --------------------------------------------------------------------- metrics
    def register_metric(self, module_id, key: str, value) -> None:
        if not hasattr(self, "_metrics"):
            self._metrics = {}
        self._metrics.setdefault(module_id, {})[key] = float(value.detach().item()) if torch.is_tensor(value) \
            else value

    def register_metrics(self, module_id, metrics_dict: Dict) -> None:
        for k, v in metrics_dict.items():
            self.register_metric(module_id, k, v)

    def compile_results(self, *, batch=None, fwd_out=None, loss_per_module=None, metrics_per_module=None) -> Dict:
        out = {}
        for mid, loss in (loss_per_module or {}).items():
            out.setdefault(mid, {})["total_loss"] = float(loss.detach().item()) if torch.is_tensor(loss) else loss
        for mid, m in (metrics_per_module or getattr(self, "_metrics", {}) or {}).items():
            out.setdefault(mid, {}).update(m)
        self._metrics = {}
        return out

    # --------------------------------------------------------------------- the generic update
    def compute_loss_for_module(self, *, module_id, config=None, batch: Dict, fwd_out: Dict) -> torch.Tensor:
        raise NotImplementedError("override compute_loss_for_module (or use the algorithm's fused update)")

    def compute_loss(self, *, fwd_out: Dict, batch: Dict) -> Dict[str, torch.Tensor]:
        out = {}
        for mid in fwd_out:
            if self.should_module_be_updated(mid):
                out[mid] = self.compute_loss_for_module(module_id=mid, config=self.cfg, batch=batch[mid],
                                                        fwd_out=fwd_out[mid])
        out[ALL_MODULES] = sum(out.values())
        return out

    def _all_optimizers(self):
        tab = self._opt_table()
        opts = [o for d in tab.values() for o in d.values()]
        return opts or [self.opt]

    def compute_gradients(self, loss_per_module: Dict, **kw) -> Dict:
        for o in self._all_optimizers():
            o.zero_grad(set_to_none=True)
        loss_per_module[ALL_MODULES].backward()
        return {id(p): p.grad for p in self.module.parameters() if p.grad is not None}

    def postprocess_gradients(self, gradients_dict: Dict) -> Dict:
        out = {}
        for mid in self._modules():
            out.update(self.postprocess_gradients_for_module(module_id=mid, config=self.cfg,
                                                             module_gradients_dict=gradients_dict))
        return out or gradients_dict

    def postprocess_gradients_for_module(self, *, module_id, config=None, module_gradients_dict: Dict) -> Dict:
        clip = (config or self.cfg).get("grad_clip")
        if clip:
            params = [p for p in self._modules()[module_id].parameters() if p.grad is not None]
            gn = torch.nn.utils.clip_grad_norm_(params, clip)
            self.register_metric(module_id, "gradients_default_optimizer_global_norm", gn)
        mod_ids = {id(p) for p in self._modules()[module_id].parameters()}
        return {k: g for k, g in module_gradients_dict.items() if k in mod_ids}

    def apply_gradients(self, gradients_dict: Dict) -> None:
        for o in self._all_optimizers():
            o.step()

    def additional_update(self, *, module_ids_to_update=None, timestep: int = 0, **kw) -> Dict:
        return {mid: self.additional_update_for_module(module_id=mid, config=self.cfg, timestep=timestep, **kw)
                for mid in (module_ids_to_update or self._modules())}

    def additional_update_for_module(self, *, module_id, config=None, timestep: int = 0, **kw) -> Dict:
        return {}

    def _custom_loss(self) -> bool:
        return type(self).compute_loss_for_module is not LearnerAPI.compute_loss_for_module

    def update_from_batch(self, batch, *, minibatch_size: Optional[int] = None, num_iters: int = 1,
                          reduce_fn=None, **kw) -> Dict:
        if not self._custom_loss():
            kind = _algo_update_kind(self.cfg)
            if kind is None or not hasattr(self, f"update_{kind}"):
                raise NotImplementedError("this learner has no compute_loss_for_module override and no "
                                          "algorithm update kind; subclass Learner or call update_<algo>")
            return getattr(self, f"update_{kind}")(batch)
        from .learner import _to_device_batch

        from ..policy.sample_batch import MultiAgentBatch

        per_module = batch.policy_batches if isinstance(batch, MultiAgentBatch) else {DEFAULT_MODULE_ID: batch}
        dev = {mid: _to_device_batch(b, self.device) for mid, b in per_module.items()}
        mods = self._modules()
        n = min(b.count for b in dev.values())
        mb = int(minibatch_size or n)
        results = {}
        for _ in range(int(num_iters)):
            perm = torch.randperm(n, device=self.device)
            for s in range(0, n, mb):
                idx = perm[s:s + mb]
                sub = {mid: {k: v[idx] for k, v in b.items() if torch.is_tensor(v) and v.shape[:1] == (b.count,)}
                       for mid, b in dev.items()}
                fwd = {mid: mods[mid].forward_train(sub[mid]) for mid in sub}
                losses = self.compute_loss(fwd_out=fwd, batch=sub)
                grads = self.compute_gradients(losses)
                grads = self.postprocess_gradients(grads)
                self.apply_gradients(grads)
                results = self.compile_results(batch=sub, fwd_out=fwd,
                                               loss_per_module={k: v for k, v in losses.items() if k != ALL_MODULES})
        self.num_updates = getattr(self, "num_updates", 0) + 1
        return results

    def update_from_episodes(self, episodes, **kw) -> Dict:
        """Episodes -> one train batch (observations, actions, rewards, terminateds per step)."""
        from ..policy.sample_batch import SampleBatch, concat_samples

        batches = []
        for ep in episodes:
            e = ep if ep.is_finalized else ep.finalize()
            n = len(e)
            batches.append(SampleBatch({"obs": np.asarray(e.get_observations(slice(0, n))),
                                        "new_obs": np.asarray(e.get_observations(slice(1, n + 1))),
                                        "actions": np.asarray(e.get_actions(slice(0, n))),
                                        "rewards": np.asarray(e.get_rewards(slice(0, n)), np.float32),
                                        "terminateds": np.asarray([False] * (n - 1) + [e.is_terminated])}))
        return self.update_from_batch(concat_samples(batches), **kw)

    def apply(self, func: Callable, *args, **kwargs):
        return func(self, *args, **kwargs)


def _algo_update_kind(cfg: Dict) -> Optional[str]:
    """The fused update an algorithm's learners run: ``_update_kind`` if set, else from the
    algorithm name the config carries (BC trains with MARWIL's update)."""
    kind = cfg.get("_update_kind") or (cfg.get("_algo") or "").lower() or None
    return {"bc": "marwil"}.get(kind, kind)


# ============================================================================ LearnerGroup
class LearnerGroupAPI:
    """Mixed into ``LearnerGroup`` (``local`` learner or a ``wg`` of learner actors)."""

    @property
    def is_local(self) -> bool:
        return self.local is not None

    @property
    def is_remote(self) -> bool:
        return self.local is None

    def foreach_learner(self, func: Callable, **kwargs) -> List[Any]:
        if self.local is not None:
            return [func(self.local, **kwargs)]
        from ..._private.worker import get

        return get([w.call.remote("apply", func) for w in self.wg.workers])

    def update_from_batch(self, batch, *, minibatch_size=None, num_iters: int = 1, async_update: bool = False,
                          **kw):
        if async_update:
            return self.async_update(batch, minibatch_size=minibatch_size, num_iters=num_iters)
        if self.local is not None:
            return self.local.update_from_batch(batch, minibatch_size=minibatch_size, num_iters=num_iters)
        kind = _algo_update_kind(self.cfg)
        if kind:
            return self.update(kind, batch)
        from ..._private.worker import get
        from .learner import _split

        shards = _split(batch, self.n)
        return get([w.call.remote("update_from_batch", s) for w, s in zip(self.wg.workers, shards)])[0]

    def update_from_episodes(self, episodes, **kw):
        if self.local is not None:
            return self.local.update_from_episodes(episodes, **kw)
        return self.foreach_learner(lambda l: l.update_from_episodes(episodes, **kw))[0]

    def async_update(self, batch, **kw):
        """Start an update in the background; returns the results of updates that finished since
        the last call (a list, possibly empty)."""
        if not hasattr(self, "_async"):
            self._async = {"thread": None, "done": [], "error": None}
        st = self._async
        if st["error"] is not None:  # the previous background update failed: surface it here
            err, st["error"] = st["error"], None
            raise err
        if st["thread"] is None or not st["thread"].is_alive():
            def run():
                try:
                    res = self.update_from_batch(batch, **kw)
                except BaseException as e:  # noqa: B036 -- handed to the caller's next call
                    st["error"] = e
                    return
                with st["lock"]:
                    st["done"].append(res)
            st.setdefault("lock", threading.Lock())
            st["thread"] = threading.Thread(target=run, daemon=True)
            st["thread"].start()
        with st.setdefault("lock", threading.Lock()):
            out, st["done"] = st["done"], []
        return out

    def additional_update(self, **kw):
        return self.foreach_learner(lambda l: l.additional_update(**kw))[0]

    def set_weights(self, weights) -> None:
        self.call("set_weights", weights)

    def get_state(self) -> Dict:
        return self.call("get_state")

    def set_state(self, state: Dict) -> None:
        if self.local is not None:
            self.local.set_state(state)
        else:
            from ..._private.worker import get

            get([w.call.remote("set_state", state) for w in self.wg.workers])

    def save_state(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        torch.save(self.get_state(), os.path.join(path, "learner_group_state.pt"))

    def load_state(self, path: str) -> None:
        self.set_state(torch.load(os.path.join(path, "learner_group_state.pt"), weights_only=True))

    def load_module_state(self, *, marl_module_ckpt_dir: Optional[str] = None, rl_module_ckpt_dirs=None,
                          module_state: Optional[Dict] = None, **kw) -> None:
        if module_state is not None:
            self.set_weights(module_state)
            return
        path = marl_module_ckpt_dir or (next(iter(rl_module_ckpt_dirs.values())) if rl_module_ckpt_dirs else None)
        if path is None:
            raise ValueError("load_module_state needs module_state or a checkpoint directory")
        self.set_weights(torch.load(os.path.join(path, "module_state.pt"), weights_only=True))

    def get_stats(self) -> Dict:
        return {"num_learners": max(1, self.n), "is_local": self.local is not None,
                "async_pending": bool(getattr(self, "_async", {}).get("thread") and self._async["thread"].is_alive())}

    def add_module(self, *, module_id, module_spec, **kw):
        return self.foreach_learner(lambda l: l.add_module(module_id=module_id, module_spec=module_spec))[0]

    def remove_module(self, module_id, **kw):
        return self.foreach_learner(lambda l: l.remove_module(module_id))[0]
