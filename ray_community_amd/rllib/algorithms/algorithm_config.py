"""AlgorithmConfig builder (reference: ``rllib/algorithms/algorithm_config.py``)."""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional


def _default_mapping_fn(agent_id, episode=None, worker=None, **kw):
    return "default_policy"


class AlgorithmConfig:
    algo_class = None

    # reference: every agent maps to the single default policy / module
    DEFAULT_POLICY_MAPPING_FN = staticmethod(_default_mapping_fn)
    DEFAULT_AGENT_TO_MODULE_MAPPING_FN = staticmethod(_default_mapping_fn)

    def __setattr__(self, k, v):
        if self.__dict__.get("_is_frozen") and k != "_is_frozen":
            raise AttributeError(f"Cannot set attribute ({k}) of an already frozen AlgorithmConfig")
        object.__setattr__(self, k, v)

    def __init__(self, algo_class=None):
        self._is_frozen = False
        if algo_class is not None:
            self.algo_class = algo_class
        # environment
        self.env = None
        self.env_config: Dict = {}
        self.observation_space = None
        self.action_space = None
        # env runners
        self.num_env_runners = 0
        self.input_ = "sampler"
        self.output = None
        self.input_config = {}
        self.output_config = {}
        self.off_policy_estimation_methods = {}
        self.num_envs_per_env_runner = 1
        self.rollout_fragment_length: Any = "auto"
        self.batch_mode = "truncate_episodes"
        self.num_cpus_per_env_runner = 1
        self.num_gpus_per_env_runner = 0  # > 0: the runner's RLModule runs its inference on that GPU share
        self.explore = True
        self.normalize_actions = False       # module acts in [-1, 1]; unsquashed to the Box bounds
        self.clip_actions = False
        self.add_default_connectors_to_env_to_module_pipeline = True
        # ConnectorV2 factories (callables; kept out of to_dict / checkpoints)
        self._env_to_module_connector = None  # (env) -> connector | [connectors]
        self._module_to_env_connector = None  # (env) -> connector | [connectors]
        self._learner_connector = None        # (obs_space, act_space) -> connector | [connectors]
        # training
        self.gamma = 0.99
        self.lr = 0.001
        self.lr_schedule = None
        self.grad_clip = None
        self.train_batch_size = 4000
        self.model: Dict = {"fcnet_hiddens": [256, 256], "fcnet_activation": "tanh", "vf_share_layers": False}
        # resources / learners
        self.num_gpus = 0
        self.num_learners = 0
        self.num_gpus_per_learner = 0
        self.framework_str = "torch"
        # evaluation
        self.evaluation_interval = None
        self.evaluation_duration = 10
        self.evaluation_duration_unit = "episodes"
        self.evaluation_num_env_runners = 0
        self.evaluation_config: Dict = {}
        # misc
        self.seed = None
        self.metrics_num_episodes_for_smoothing = 100
        # multi-agent
        self.policies = None                 # {policy_id: None | PolicySpec | (cls, obs_space, act_space, cfg)}
        self.policy_mapping_fn = None        # (agent_id, episode, worker, **kw) -> policy_id
        self.policies_to_train = None
        self.min_sample_timesteps_per_iteration = 0
        # fault tolerance (reference algorithm_config.py:486-499, fault_tolerance():2673)
        self.ignore_env_runner_failures = False
        self.recreate_failed_env_runners = False
        self.max_num_env_runner_restarts = 1000
        self.delay_between_env_runner_restarts_s = 60.0
        self.restart_failed_sub_environments = False
        self.num_consecutive_env_runner_failures_tolerance = 100
        self.env_runner_health_probe_timeout_s = 30.0
        self.env_runner_restore_timeout_s = 1800.0
        # checkpointing (reference checkpointing():2596)
        self.export_native_model_files = False
        self.checkpoint_trainable_policies_only = False
        # custom RLModule (reference rl_module():2737)
        self._rl_module_spec = None
        # exploration / experimental / python environment (reference exploration():2141,
        # experimental():2806, python_environment():1431)
        self.exploration_config: Dict = {}
        self._experimental: Dict = {}
        self.extra_python_environs_for_driver: Dict = {}
        self.extra_python_environs_for_worker: Dict = {}
        self.train_batch_size_per_learner = None
        self.in_evaluation = False
        self._per_module_overrides: Dict = {}

    # ------------------------------------------------------------------ builder methods
    def environment(self, env=None, *, env_config=None, observation_space=None, action_space=None, **kw):
        if env is not None:
            self.env = env
        if env_config is not None:
            self.env_config = dict(env_config)
        self.observation_space = observation_space or self.observation_space
        self.action_space = action_space or self.action_space
        return self

    def env_runners(self, *, num_env_runners=None, num_envs_per_env_runner=None, rollout_fragment_length=None,
                    batch_mode=None, num_cpus_per_env_runner=None, num_gpus_per_env_runner=None, explore=None,
                    env_to_module_connector=None, module_to_env_connector=None,
                    add_default_connectors_to_env_to_module_pipeline=None, normalize_actions=None,
                    clip_actions=None, **kw):
        """``env_to_module_connector(env)`` / ``module_to_env_connector(env)``: return a ConnectorV2,
        a list of them or a pipeline (rllib/connectors)."""
        for k, v in dict(num_env_runners=num_env_runners, num_envs_per_env_runner=num_envs_per_env_runner,
                         rollout_fragment_length=rollout_fragment_length, batch_mode=batch_mode,
                         num_cpus_per_env_runner=num_cpus_per_env_runner,
                         num_gpus_per_env_runner=num_gpus_per_env_runner, explore=explore,
                         add_default_connectors_to_env_to_module_pipeline=add_default_connectors_to_env_to_module_pipeline,
                         normalize_actions=normalize_actions, clip_actions=clip_actions).items():
            if v is not None:
                setattr(self, k, v)
        if env_to_module_connector is not None:
            self._env_to_module_connector = env_to_module_connector
        if module_to_env_connector is not None:
            self._module_to_env_connector = module_to_env_connector
        unknown = set(kw) - {"sample_timeout_s", "num_gpus_per_env_runner", "create_env_on_local_worker",
                             "observation_filter", "compress_observations", "remote_worker_envs",
                             "remote_env_batch_wait_ms", "validate_env_runners_after_construction",
                             "episode_lookback_horizon", "use_worker_filter_stats", "update_worker_filter_stats",
                             "gym_env_vectorize_mode"}
        if unknown:
            raise TypeError(f"env_runners() got unsupported argument(s) {sorted(unknown)}")
        return self

    def rollouts(self, *, num_rollout_workers=None, num_envs_per_worker=None, rollout_fragment_length=None,
                 batch_mode=None, **kw):
        return self.env_runners(num_env_runners=num_rollout_workers, num_envs_per_env_runner=num_envs_per_worker,
                                rollout_fragment_length=rollout_fragment_length, batch_mode=batch_mode)

    def training(self, **kw):
        """Algorithm hyperparameters; ``learner_connector(obs_space, act_space)`` returns learner
        ConnectorV2 piece(s) run on the train batch before the loss."""
        aliases = {"sgd_minibatch_size": "minibatch_size", "num_sgd_iter": "num_epochs", "lambda": "lambda_"}
        if kw.get("learner_connector") is not None:
            self._learner_connector = kw.pop("learner_connector")
        kw.pop("learner_connector", None)
        for k, v in kw.items():
            k = aliases.get(k, k)
            if k == "model" and v is not None:
                m = dict(self.model)
                m.update(v)
                self.model = m
                continue
            setattr(self, k, v)
        return self

    def resources(self, *, num_gpus=None, num_cpus_for_main_process=None, **kw):
        if num_gpus is not None:
            self.num_gpus = num_gpus
        return self

    def learners(self, *, num_learners=None, num_gpus_per_learner=None, **kw):
        if num_learners is not None:
            self.num_learners = num_learners
        if num_gpus_per_learner is not None:
            self.num_gpus_per_learner = num_gpus_per_learner
        return self

    def framework(self, framework="torch", **kw):
        if framework not in ("torch", None):
            raise ValueError("only the torch framework is supported on MI355X")
        self.framework_str = "torch"
        return self

    def evaluation(self, *, evaluation_interval=None, evaluation_duration=None, evaluation_duration_unit=None,
                   evaluation_num_env_runners=None, evaluation_config=None, off_policy_estimation_methods=None, **kw):
        """``off_policy_estimation_methods``: {name: {"type": ImportanceSampling | ..., **kwargs}}:
        ``evaluate()`` then also estimates the current policy's value from the offline input."""
        for k, v in dict(evaluation_interval=evaluation_interval, evaluation_duration=evaluation_duration,
                         evaluation_duration_unit=evaluation_duration_unit,
                         evaluation_num_env_runners=evaluation_num_env_runners,
                         evaluation_config=evaluation_config,
                         off_policy_estimation_methods=off_policy_estimation_methods).items():
            if v is not None:
                setattr(self, k, v)
        return self

    def debugging(self, *, seed=None, **kw):
        if seed is not None:
            self.seed = seed
        return self

    def reporting(self, *, metrics_num_episodes_for_smoothing=None, min_sample_timesteps_per_iteration=None, **kw):
        if metrics_num_episodes_for_smoothing is not None:
            self.metrics_num_episodes_for_smoothing = metrics_num_episodes_for_smoothing
        if min_sample_timesteps_per_iteration is not None:
            self.min_sample_timesteps_per_iteration = min_sample_timesteps_per_iteration
        return self

    def rl_module(self, *, model_config=None, model_config_dict=None, rl_module_spec=None, **kw):
        """``model_config``: network settings merged into ``model``; ``rl_module_spec``: an
        ``RLModuleSpec`` (custom ``module_class`` built with (obs_space, act_space, model_config))
        or, multi-agent, a ``MultiRLModuleSpec`` / {module_id: RLModuleSpec}."""
        m = model_config or model_config_dict
        if m:
            self.model = {**self.model, **dict(m)}
        if rl_module_spec is not None:
            self._rl_module_spec = rl_module_spec
        return self

    @property
    def rl_module_spec(self):
        return self._rl_module_spec

    def fault_tolerance(self, *, recreate_failed_env_runners=None, ignore_env_runner_failures=None,
                        max_num_env_runner_restarts=None, delay_between_env_runner_restarts_s=None,
                        restart_failed_sub_environments=None, num_consecutive_env_runner_failures_tolerance=None,
                        env_runner_health_probe_timeout_s=None, env_runner_restore_timeout_s=None,
                        recreate_failed_workers=None, ignore_worker_failures=None, max_num_worker_restarts=None,
                        delay_between_worker_restarts_s=None, num_consecutive_worker_failures_tolerance=None,
                        worker_health_probe_timeout_s=None, worker_restore_timeout_s=None,
                        restart_failed_env_runners=None, **kw):
        """Env-runner fault tolerance (reference ``fault_tolerance``, old ``*_worker*`` names
        accepted): ``recreate_failed_env_runners`` replaces a dead runner with a fresh actor of the
        same index (restored with the current weights before it samples again);
        ``ignore_env_runner_failures`` drops it and goes on with the healthy ones."""
        def pick(*vals):
            for v in vals:
                if v is not None:
                    return v
            return None

        vals = {
            "recreate_failed_env_runners": pick(recreate_failed_env_runners, restart_failed_env_runners,
                                                recreate_failed_workers),
            "ignore_env_runner_failures": pick(ignore_env_runner_failures, ignore_worker_failures),
            "max_num_env_runner_restarts": pick(max_num_env_runner_restarts, max_num_worker_restarts),
            "delay_between_env_runner_restarts_s": pick(delay_between_env_runner_restarts_s,
                                                        delay_between_worker_restarts_s),
            "restart_failed_sub_environments": restart_failed_sub_environments,
            "num_consecutive_env_runner_failures_tolerance": pick(num_consecutive_env_runner_failures_tolerance,
                                                                  num_consecutive_worker_failures_tolerance),
            "env_runner_health_probe_timeout_s": pick(env_runner_health_probe_timeout_s, worker_health_probe_timeout_s),
            "env_runner_restore_timeout_s": pick(env_runner_restore_timeout_s, worker_restore_timeout_s),
        }
        for k, v in vals.items():
            if v is not None:
                setattr(self, k, v)
        if kw:
            raise TypeError(f"fault_tolerance() got unsupported argument(s) {sorted(kw)}")
        return self

    # old-stack attribute names
    @property
    def recreate_failed_workers(self):
        return self.recreate_failed_env_runners

    @property
    def ignore_worker_failures(self):
        return self.ignore_env_runner_failures

    def checkpointing(self, *, export_native_model_files=None, checkpoint_trainable_policies_only=None, **kw):
        """``checkpoint_trainable_policies_only``: multi-agent checkpoints hold only the policies
        in ``policies_to_train``; ``export_native_model_files``: each checkpoint also gets every
        policy's ``model.pt`` (a ``weights_only``-loadable ``state_dict``)."""
        if export_native_model_files is not None:
            self.export_native_model_files = bool(export_native_model_files)
        if checkpoint_trainable_policies_only is not None:
            self.checkpoint_trainable_policies_only = bool(checkpoint_trainable_policies_only)
        return self

    def validate(self) -> None:
        """Reject inconsistent settings before anything is built (reference ``validate``,
        ``algorithm_config.py:791``). Algorithm configs extend it with their own checks."""
        def bad(msg):
            raise ValueError(msg)

        if self.framework_str != "torch":
            bad("only the torch framework is supported")
        if int(self.num_env_runners) < 0:
            bad(f"num_env_runners must be >= 0, got {self.num_env_runners}")
        if int(self.num_envs_per_env_runner) < 1:
            bad(f"num_envs_per_env_runner must be >= 1, got {self.num_envs_per_env_runner}")
        rfl = self.rollout_fragment_length
        if rfl != "auto" and (not isinstance(rfl, int) or rfl <= 0):
            bad(f"rollout_fragment_length must be 'auto' or a positive int, got {rfl!r}")
        if self.batch_mode not in ("truncate_episodes", "complete_episodes"):
            bad(f"batch_mode must be 'truncate_episodes' or 'complete_episodes', got {self.batch_mode!r}")
        if not (0.0 <= float(self.gamma) <= 1.0):
            bad(f"gamma must be in [0, 1], got {self.gamma}")
        if self.lr is not None and self.lr_schedule is None and float(self.lr) <= 0:
            bad(f"lr must be > 0, got {self.lr}")
        if int(self.train_batch_size) <= 0:
            bad(f"train_batch_size must be > 0, got {self.train_batch_size}")
        if int(self.num_learners) < 0 or float(self.num_gpus_per_learner) < 0:
            bad("num_learners and num_gpus_per_learner must be >= 0")
        if self.evaluation_duration_unit not in ("episodes", "timesteps"):
            bad(f"evaluation_duration_unit must be 'episodes' or 'timesteps', got {self.evaluation_duration_unit!r}")
        if self.evaluation_interval is not None and int(self.evaluation_interval) < 0:
            bad("evaluation_interval must be >= 0 or None")
        if self.policies:
            if self.policy_mapping_fn is not None and not callable(self.policy_mapping_fn):
                bad("policy_mapping_fn must be callable")
            unknown = set(self.policies_to_train or ()) - set(self.policies)
            if unknown and not callable(self.policies_to_train):
                bad(f"policies_to_train names unknown policies {sorted(unknown)}")
        if int(self.max_num_env_runner_restarts) < 0 or float(self.delay_between_env_runner_restarts_s) < 0:
            bad("max_num_env_runner_restarts and delay_between_env_runner_restarts_s must be >= 0")
        if (self.model or {}).get("use_lstm") and int((self.model or {}).get("max_seq_len", 20)) <= 0:
            bad("model.max_seq_len must be > 0 with use_lstm")

    def api_stack(self, **kw):
        return self

    def multi_agent(self, *, policies=None, policy_mapping_fn=None, policies_to_train=None, **kw):
        """Several policies, each with its own RLModule and learner group; agents are bound to
        policies by ``policy_mapping_fn(agent_id, episode, worker)`` (reference:
        ``AlgorithmConfig.multi_agent``). ``policies`` may be a set/list of ids or a dict of ids to
        ``None`` / ``PolicySpec`` / ``(cls, obs_space, act_space, config)``."""
        if policies is not None:
            self.policies = {p: None for p in policies} if isinstance(policies, (set, list, tuple)) else dict(policies)
        if policy_mapping_fn is not None:
            self.policy_mapping_fn = policy_mapping_fn
        if policies_to_train is not None:
            self.policies_to_train = list(policies_to_train)
        return self

    @property
    def is_multi_agent(self) -> bool:
        from ..env.multi_agent_env import MultiAgentEnv, _MA_REGISTRY

        if self.policies:
            return True
        e = self.env
        return (isinstance(e, str) and e in _MA_REGISTRY) or isinstance(e, MultiAgentEnv) or \
            (isinstance(e, type) and issubclass(e, MultiAgentEnv))

    def offline_data(self, *, input_=None, output=None, input_config=None, output_config=None, **kw):
        """``input_``: directory / glob of JSON batches for offline algorithms (BC, MARWIL);
        ``output``: directory the env runners write their sampled batches to."""
        if input_ is not None:
            self.input_ = input_
        if output is not None:
            self.output = output
        if input_config is not None:
            self.input_config = dict(input_config)
        if output_config is not None:
            self.output_config = dict(output_config)
        return self

    def callbacks(self, callbacks_class=None, **kw):
        """A ``DefaultCallbacks`` subclass (or a list of them, see ``make_multi_callbacks``)."""
        self._callbacks = callbacks_class if callbacks_class is not None else kw.get("cb")
        return self

    @property
    def callbacks_class(self):
        return getattr(self, "_callbacks", None)

    @callbacks_class.setter
    def callbacks_class(self, v):
        self._callbacks = v

    def exploration(self, *, explore=None, exploration_config=None, **kw):
        if explore is not None:
            self.explore = bool(explore)
        if exploration_config is not None:
            self.exploration_config = {**self.exploration_config, **dict(exploration_config)}
        return self

    def experimental(self, **kw):
        """Experimental switches (``_torch_grad_scaler_class``, ``_tf_policy_handles_more_than_one_loss``,
        ...): stored under their names; unknown ones are kept too, as in the reference."""
        self._experimental.update(kw)
        return self

    def python_environment(self, *, extra_python_environs_for_driver=None, extra_python_environs_for_worker=None):
        """Environment variables set in the driver / every env runner process."""
        if extra_python_environs_for_driver is not None:
            self.extra_python_environs_for_driver = dict(extra_python_environs_for_driver)
        if extra_python_environs_for_worker is not None:
            self.extra_python_environs_for_worker = dict(extra_python_environs_for_worker)
        return self

    @classmethod
    def overrides(cls, **kwargs) -> Dict:
        """A dict of setting overrides (for ``evaluation(evaluation_config=...)`` and per-module
        overrides), checked against the config's attribute names."""
        default = cls()
        for k in kwargs:
            if not hasattr(default, k) and k != "lambda":
                raise KeyError(f"Invalid property name {k!r} for config class {cls.__name__}")
        return dict(kwargs)

    # ------------------------------------------------------------------ derived views
    @property
    def num_workers(self) -> int:  # old-stack name of num_env_runners
        return self.num_env_runners

    @property
    def uses_new_env_runners(self) -> bool:
        return True

    @property
    def total_train_batch_size(self) -> int:
        """The batch one training iteration learns from: per-learner size x learners, or
        ``train_batch_size``."""
        if self.train_batch_size_per_learner:
            return int(self.train_batch_size_per_learner) * max(1, int(self.num_learners))
        return int(self.train_batch_size)

    @property
    def is_atari(self) -> bool:
        e = self.env
        if isinstance(e, str) and (e.startswith("ALE/") or "NoFrameskip" in e or "Atari" in e):
            return True
        shp = getattr(self.observation_space, "shape", None)
        return bool(shp) and tuple(shp)[:2] == (84, 84)

    @property
    def multiagent(self) -> Dict:
        """Old-stack dict view of the multi-agent settings."""
        return {"policies": self.policies, "policy_mapping_fn": self.policy_mapping_fn,
                "policies_to_train": self.policies_to_train}

    @property
    def learner_class(self):
        return self.get_default_learner_class()

    def get_default_learner_class(self):
        from ..core.learner import Learner

        return Learner

    def get_default_rl_module_spec(self):
        from ..core.rl_module import RecurrentRLModule, RLModule, RLModuleSpec

        m = self.model or {}
        return RLModuleSpec(module_class=RecurrentRLModule if m.get("use_lstm") else RLModule, model_config=dict(m))

    def get_multi_agent_setup(self, *, env=None, spaces=None):
        """(policies {id: PolicySpec-like tuple}, is_policy_to_train(policy_id) callable)."""
        pols = dict(self.policies) if self.policies else {"default_policy": None}
        if spaces:
            pols = {p: (v if v is not None else (None, *spaces.get(p, (None, None)), {})) for p, v in pols.items()}
        ptt = self.policies_to_train

        def is_policy_to_train(pid, batch=None):
            if ptt is None:
                return True
            return ptt(pid, batch) if callable(ptt) else pid in ptt

        return pols, is_policy_to_train

    def get_marl_module_spec(self, *, policy_dict=None, single_agent_rl_module_spec=None, env=None, spaces=None):
        """The MultiRLModuleSpec of this config: one spec per policy (a user ``rl_module_spec`` per
        module id wins, else the default module spec)."""
        from ..core.rl_module import MultiRLModuleSpec, RLModuleSpec

        user = self._rl_module_spec
        if isinstance(user, MultiRLModuleSpec):
            return user
        pols = policy_dict or self.get_multi_agent_setup(spaces=spaces)[0]
        base = single_agent_rl_module_spec or self.get_default_rl_module_spec()
        specs = {}
        for pid in pols:
            spec = user.get(pid) if isinstance(user, dict) else (user if isinstance(user, RLModuleSpec) else None)
            if spec is None:
                spec = RLModuleSpec(base.module_class, model_config=dict(base.model_config))
                if spaces and pid in spaces:
                    spec.observation_space, spec.action_space = spaces[pid]
            specs[pid] = spec
        return MultiRLModuleSpec(specs)

    get_multi_rl_module_spec = get_marl_module_spec

    def get_config_for_module(self, module_id):
        """A copy of this config with the overrides registered for ``module_id`` applied."""
        c = self.copy(copy_frozen=False)
        for k, v in (self._per_module_overrides.get(module_id) or {}).items():
            setattr(c, k, v)
        return c

    def get_evaluation_config_object(self):
        """The config evaluation runs with: a copy with ``evaluation_config`` applied, ``in_evaluation``
        set and the evaluation runner count as ``num_env_runners``."""
        c = self.copy(copy_frozen=False)
        ov = self.evaluation_config
        if isinstance(ov, AlgorithmConfig):
            ov = {k: v for k, v in ov.to_dict().items() if k != "framework"}
        c.update_from_dict(dict(ov or {}))
        c.in_evaluation = True
        c.num_env_runners = self.evaluation_num_env_runners
        return c

    def get_torch_compile_worker_config(self) -> Dict:
        """No tracing compiler on this stack (HIP graphs and hand-written kernels instead): the
        compile config is reported disabled."""
        return {"torch_compile": False, "torch_compile_backend": None, "torch_compile_mode": None}

    def validate_train_batch_size_vs_rollout_fragment_length(self) -> None:
        """A fixed rollout_fragment_length must let the runners fill train_batch_size within a
        factor of 10 (reference check of the same name)."""
        if self.rollout_fragment_length == "auto" or self.batch_mode != "truncate_episodes":
            return
        per_round = int(self.rollout_fragment_length) * max(1, int(self.num_env_runners)) * \
            int(self.num_envs_per_env_runner)
        tbs = self.total_train_batch_size
        if tbs > 0 and (per_round > 10 * tbs or per_round * 10 < tbs and tbs % per_round != 0 and per_round < tbs // 10):
            raise ValueError(f"rollout_fragment_length ({self.rollout_fragment_length}) x runners x envs "
                             f"({per_round} per round) does not fit train_batch_size ({tbs})")

    # ------------------------------------------------------------------ component builders
    def build_env_to_module_connector(self, env):
        from ..connectors import build_env_to_module

        return build_env_to_module(dict(self.to_dict(), **self._connector_dict()), env)

    def build_module_to_env_connector(self, env):
        from ..connectors import build_module_to_env

        return build_module_to_env(dict(self.to_dict(), **self._connector_dict()), env)

    def build_learner_connector(self, input_observation_space, input_action_space, device=None):
        from ..connectors import build_learner_connector

        return build_learner_connector(dict(self.to_dict(), **self._connector_dict()), input_observation_space,
                                       input_action_space)

    def _learner_config(self) -> Dict:
        d = self.to_dict()
        d.update(self._connector_dict())
        if self.algo_class is not None:
            d["_algo"] = getattr(self.algo_class, "__name__", None)
        return d

    def build_learner(self, *, env=None, spaces=None, observation_space=None, action_space=None, use_gpu=False):
        """One Learner (RLModule + optimizer + learner connector) for this config."""
        obs, act = self._spaces(env, spaces, observation_space, action_space)
        return self.get_default_learner_class()(self._learner_config(), obs, act, use_gpu)

    def build_learner_group(self, *, env=None, spaces=None, observation_space=None, action_space=None):
        """The LearnerGroup an Algorithm trains with (local learner, or ``num_learners`` GPU learner
        actors over one RCCL process group)."""
        from ..core.learner import LearnerGroup

        obs, act = self._spaces(env, spaces, observation_space, action_space)
        return LearnerGroup(self._learner_config(), obs, act)

    def _spaces(self, env, spaces, obs, act):
        if spaces:
            obs, act = next(iter(spaces.values())) if isinstance(spaces, dict) else spaces
        if (obs is None or act is None) and env is not None:
            obs, act = env.observation_space, env.action_space
        obs, act = obs or self.observation_space, act or self.action_space
        if obs is None or act is None:
            from ..env.envs import make_vector_env

            e = make_vector_env(self.env, 1, self.env_config)
            obs, act = e.observation_space, e.action_space
        return obs, act

    # ------------------------------------------------------------------ misc
    def freeze(self) -> None:
        """No further changes (the Algorithm freezes the config it runs with)."""
        self._is_frozen = True

    def copy(self, copy_frozen=None):
        c = copy.deepcopy(self)
        if copy_frozen is not True:
            c._is_frozen = False
        return c

    def keys(self):
        return self.to_dict().keys()

    def values(self):
        return self.to_dict().values()

    def items(self):
        return self.to_dict().items()

    def pop(self, k, default=None):
        """Reset ``k`` to the default config's value and return the current one."""
        v = getattr(self, k, default)
        if hasattr(type(self)(), k):
            setattr(self, k, getattr(type(self)(), k))
        return v

    def serialize(self) -> Dict:
        """A JSON-able dict of the config: classes and callables by import path / name."""
        import json

        def conv(v):
            if isinstance(v, (str, int, float, bool)) or v is None:
                return v
            if isinstance(v, dict):
                return {str(k): conv(x) for k, x in v.items()}
            if isinstance(v, (list, tuple, set)):
                return [conv(x) for x in v]
            if isinstance(v, type) or callable(v):
                return f"{getattr(v, '__module__', '?')}.{getattr(v, '__qualname__', repr(v))}"
            try:
                json.dumps(v)
                return v
            except TypeError:
                return repr(v)

        return {k: conv(v) for k, v in self.to_dict().items()}

    def to_dict(self) -> Dict:
        d = {k: v for k, v in self.__dict__.items() if not k.startswith("_")}
        d.pop("in_evaluation", None) if not self.__dict__.get("in_evaluation") else None
        d["framework"] = self.framework_str
        return d

    # old-stack config keys (tuned-example YAML files, ``rllib train --config``) -> current names
    _LEGACY_KEYS = {"lambda": "lambda_", "num_workers": "num_env_runners", "num_rollout_workers": "num_env_runners",
                    "num_envs_per_worker": "num_envs_per_env_runner", "num_sgd_iter": "num_epochs",
                    "sgd_minibatch_size": "minibatch_size", "evaluation_num_workers": "evaluation_num_env_runners"}
    _IGNORED_KEYS = ("framework", "eager_tracing", "log_level", "create_env_on_driver")

    def update_from_dict(self, d: Dict):
        for k, v in d.items():
            if k in self._IGNORED_KEYS:
                continue
            k = self._LEGACY_KEYS.get(k, k)
            if k == "model" and isinstance(v, dict):
                m = dict(self.model or {})
                m.update(v)
                v = m
            setattr(self, k, v)
        return self

    @classmethod
    def from_dict(cls, d):
        return cls().update_from_dict(d)

    def get_rollout_fragment_length(self):
        if self.rollout_fragment_length == "auto":
            n = max(1, self.num_env_runners) * self.num_envs_per_env_runner
            return max(1, self.train_batch_size // n)
        return int(self.rollout_fragment_length)

    def build(self, env=None, logger_creator=None, use_copy=True):
        if env is not None:
            self.env = env
        self.validate()
        return self.algo_class(config=self.copy() if use_copy else self)

    build_algo = build

    def __getitem__(self, k):
        return getattr(self, k)

    def get(self, k, default=None):
        return getattr(self, k, default)

    def runner_dict(self) -> Dict:
        d = self.to_dict()
        d["rollout_fragment_length"] = self.get_rollout_fragment_length()
        d["callbacks_class"] = getattr(self, "_callbacks", None)
        d.update(self._connector_dict())
        return d

    def _connector_dict(self) -> Dict:
        return {"env_to_module_connector": self._env_to_module_connector,
                "module_to_env_connector": self._module_to_env_connector,
                "learner_connector": self._learner_connector,
                "rl_module_spec": self._rl_module_spec}
