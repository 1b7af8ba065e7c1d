"""Env runners (reference: ``rllib/env/single_agent_env_runner.py``, ``evaluation/rollout_worker.py``).

Each runner owns a natively vectorised env (N sub-envs stepped as one numpy batch) and a CPU
copy of the RLModule; it returns rollout fragments as env-major ``[N, T]`` column blocks with
the value bootstraps needed for exact GAE under auto-reset and truncation (``next_vf_preds``).
Observations pass through the env-to-module ConnectorV2 pipeline and actions through the
module-to-env pipeline (``rllib/connectors``); the fragment stores what the module saw.
Recurrent modules (``model.use_lstm``): one ``(h, c)`` row per sub-env, zeroed at episode
starts; the state each step entered with is stored (``state_in``) with the episode-start flags
(``is_first``) so the learner can replay the recurrence.
"""
from __future__ import annotations

import collections
import time
from typing import Dict, Optional

import numpy as np
import torch

from ..core.rl_module import make_module
from ..policy.sample_batch import SampleBatch
from .envs import make_vector_env


class EnvRunner:
    def __init__(self, config: Dict, worker_index: int = 0):
        torch.set_num_threads(int(config.get("num_cpus_per_env_runner_threads", 1)))
        self.cfg = config
        self.worker_index = worker_index
        seed = config.get("seed")
        self.seed = None if seed is None else int(seed) + 1000 * worker_index
        if self.seed is not None:
            torch.manual_seed(self.seed)
        from .env_context import EnvContext

        self.env_context = EnvContext(config.get("env_config") or {}, worker_index=worker_index,
                                      remote=worker_index > 0, num_workers=config.get("num_env_runners", 0))
        self.env = make_vector_env(config["env"], config.get("num_envs_per_env_runner", 1), self.env_context,
                                   seed=self.seed)
        self.N = self.env.num_envs
        from ..connectors import VectorEnvContext, build_env_to_module, build_module_to_env

        self.env_to_module = build_env_to_module(config, self.env)
        self.module_to_env = build_module_to_env(config, self.env)
        self.has_stateful_connectors = len(self.env_to_module) > 0
        self._ctx = VectorEnvContext(self.N)
        self._pending_mobs = None  # connector output for self.obs computed at the previous fragment's end
        self._module_obs_space = self.env_to_module.observation_space
        fs = int(config.get("episode_frame_stack", 1) or 1)
        if fs > 1:  # episode-path frame stacking: the module sees fs observations concatenated
            from ..utils.spaces import Box

            sp = self._module_obs_space
            self._module_obs_space = Box(np.concatenate([np.asarray(sp.low, np.float32)] * fs, -1),
                                         np.concatenate([np.asarray(sp.high, np.float32)] * fs, -1),
                                         dtype=np.float32)
        self.module = make_module(config, self._module_obs_space, self.env.action_space)
        self.module.eval()
        self.stateful = bool(getattr(self.module, "is_stateful", False))
        # per-phase wall time of sample() (``profile_env_runner`` config / bench_rllib.py
        # --profile-runner): env-to-module connectors, policy inference (+ device->host copy),
        # module-to-env connectors, env.step, per-step bookkeeping, fragment assembly
        self._prof = {} if config.get("profile_env_runner") else None
        # GPU inference (num_gpus_per_env_runner > 0): the module lives on the runner's GPU share,
        # observations go up once per step and ONE packed [N, 3 + A] tensor comes back
        self.device = torch.device("cpu")
        if float(config.get("num_gpus_per_env_runner", 0) or 0) > 0 and torch.cuda.is_available():
            self.device = torch.device("cuda", torch.cuda.current_device())
            self.module.to(self.device)
        self.obs, _ = self.env.reset(seed=self.seed)
        if self.device.type == "cpu" and getattr(self.module, "is_image", False):
            # the module's input is the runner's HWC frames permuted, i.e. channels-last memory:
            # channels-last conv weights keep oneDNN on its NHWC path with no per-call reorder
            # (CPU inference 1.54 vs 1.63 ms per 16-env step, scripts/runner_infer_bench.py);
            # load_state_dict copies into the existing parameters, so the format survives weight syncs
            self.module.to(memory_format=torch.channels_last)
        self._rstate = self.module.get_initial_state(self.N, self.device) if self.stateful else None
        self.ep_ret = np.zeros(self.N)
        self.ep_len = np.zeros(self.N, dtype=np.int64)
        self.completed = collections.deque(maxlen=int(config.get("metrics_num_episodes_for_smoothing", 100)))
        self.new_episodes = []
        self.steps_sampled = 0
        self.weights_version = -1
        self._rng = np.random.default_rng(self.seed)
        from ..algorithms.callbacks import Episode, build, overrides

        self._Episode = Episode
        self.callbacks = build(config.get("callbacks_class"))
        self._cb_step = overrides(self.callbacks, "on_episode_step")
        self.new_custom_metrics = []
        if self.callbacks is not None:
            self.callbacks.on_environment_created(env_runner=self, env=self.env, env_context=self.env_context)
            self._eps = [Episode(i) for i in range(self.N)]
            for i, ep in enumerate(self._eps):
                self.callbacks.on_episode_start(episode=ep, env_runner=self, env_index=i)

    def spaces(self):
        """(module observation space = the env-to-module pipeline's output, frame-stacked on the
        episode path; action space)."""
        return self._module_obs_space, self.env.action_space

    # ------------------------------------------------------------------ connectors
    def get_connector_state(self):
        return self.env_to_module.get_state()

    def set_connector_state(self, state):
        self.env_to_module.set_state(state)
        return True

    def _module_obs(self, obs, explore):
        """env obs [N, ...] -> module input through the env-to-module pipeline (advances its state)."""
        if not len(self.env_to_module):
            return obs
        return self.env_to_module(rl_module=self.module, batch={"obs": obs}, episodes=self._ctx, explore=explore,
                                  shared_data={})["obs"]

    def _peek_obs(self, obs, idx, actions, rewards):
        """Module input for sub-envs ``idx`` observing ``obs`` after ``actions`` / ``rewards``,
        without committing connector state (final observations of truncated episodes)."""
        if not len(self.env_to_module):
            return obs
        ctx = self._ctx.subset(idx, actions, rewards)
        return self.env_to_module(rl_module=self.module, batch={"obs": obs}, episodes=ctx, explore=False,
                                  shared_data={"peek": True})["obs"]

    def _env_actions(self, an, explore):
        if not len(self.module_to_env):
            return an
        return self.module_to_env(rl_module=self.module, batch={"actions": an, "actions_for_env": an.copy()},
                                  episodes=self._ctx, explore=explore, shared_data={})["actions_for_env"]

    def set_weights(self, state, version: int = 0):
        if version != self.weights_version:
            self.module.set_state(state)
            self.weights_version = version
        return True

    def get_weights(self):
        return self.module.get_state()

    def _track(self, rew, term, trunc, info=None):
        self.ep_ret += rew
        self.ep_len += 1
        done = term | trunc
        cb = self.callbacks
        if cb is not None and self._cb_step:
            for i, ep in enumerate(self._eps):
                ep.total_reward, ep.length, ep.last_info = float(self.ep_ret[i]), int(self.ep_len[i]), info
                cb.on_episode_step(episode=ep, env_runner=self, env_index=i)
        if done.any():
            for i in np.nonzero(done)[0]:
                ep = (float(self.ep_ret[i]), int(self.ep_len[i]))
                self.completed.append(ep)
                self.new_episodes.append(ep)
                if cb is not None:
                    e = self._eps[i]
                    e.total_reward, e.length = ep
                    cb.on_episode_end(episode=e, env_runner=self, env_index=int(i))
                    if e.custom_metrics:
                        self.new_custom_metrics.append(dict(e.custom_metrics))
                    self._eps[i] = self._Episode(int(i))
                    cb.on_episode_start(episode=self._eps[i], env_runner=self, env_index=int(i))
            self.ep_ret[done] = 0
            self.ep_len[done] = 0

    def _to_host(self, a, lp, v, logits):
        """One device->host copy per step for the policy outputs (discrete actions travel as f32)."""
        if a.dim() != 1 or a.dtype not in (torch.int64, torch.int32):
            return a.cpu(), lp.cpu(), v.cpu(), None if logits is None else logits.cpu()
        cols = [a.float().unsqueeze(1), lp.float().unsqueeze(1), v.float().unsqueeze(1)]
        if logits is not None:
            cols.append(logits.float())
        h = torch.cat(cols, 1).cpu()
        return h[:, 0].long(), h[:, 1], h[:, 2], (h[:, 3:] if logits is not None else None)

    def _value(self, obs, state=None):
        o = torch.from_numpy(np.ascontiguousarray(obs))
        if self.device.type == "cuda":
            o = o.to(self.device, non_blocking=True)
        if self.stateful:
            return self.module.forward_step(o, state)[1].float().cpu().numpy()
        return self.module.forward(o)[1].float().cpu().numpy()

    @torch.no_grad()
    def sample(self, num_steps: Optional[int] = None, explore: bool = True) -> SampleBatch:
        """On-policy fragment of T = num_steps // N steps per sub-env (PPO / IMPALA)."""
        T = max(1, int(num_steps or self.cfg.get("rollout_fragment_length", 64) * self.N) // self.N)
        N = self.N
        dist = getattr(self.module, "dist_cls", None)  # None: SAC-style module with its own squashed policy
        act_shape = () if dist is not None and dist.__name__ == "Categorical" else self.env.action_space.shape
        acts = np.empty((N, T) + tuple(act_shape), dtype=np.int64 if act_shape == () else np.float32)
        logp = np.empty((N, T), dtype=np.float32)
        vf = np.empty((N, T), dtype=np.float32)
        rew = np.empty((N, T), dtype=np.float32)
        term = np.empty((N, T), dtype=bool)
        trunc = np.empty((N, T), dtype=bool)
        first_buf = np.empty((N, T), dtype=bool)
        eid_buf = np.empty((N, T), dtype=np.int64)
        if getattr(self, "_eps_ids", None) is None:  # running episode ids, unique per runner and sub-env
            self._eps_ids = np.arange(N, dtype=np.int64) + ((int(self.worker_index) + 1) << 40)
            self._eps_next = int(self._eps_ids.max()) + 1
        obs_buf = logits_buf = state_buf = None
        trunc_fix = []  # (t, env indices, module-input final obs, state after the step)
        gpu = self.device.type == "cuda"
        ctx = self._ctx
        prof = self._prof
        clk = time.perf_counter
        t_start = clk()
        for t in range(T):
            if prof is not None:
                t0 = clk()
            if self._pending_mobs is not None:
                mobs, self._pending_mobs = self._pending_mobs, None
            else:
                mobs = self._module_obs(self.obs, explore)
            if prof is not None:
                t1 = clk()
                prof["env_to_module_s"] = prof.get("env_to_module_s", 0.0) + (t1 - t0)
            if obs_buf is None:
                obs_buf = np.empty((N, T) + mobs.shape[1:], dtype=mobs.dtype)
            first_buf[:, t] = ctx.is_first
            o = torch.from_numpy(np.ascontiguousarray(mobs))
            if gpu:
                o = o.to(self.device, non_blocking=True)
            if self.stateful:
                if ctx.is_first.any():
                    self._rstate[torch.from_numpy(ctx.is_first).to(self._rstate.device)] = 0.0
                if state_buf is None:
                    state_buf = np.empty((N, T, self._rstate.shape[1]), dtype=np.float32)
                state_buf[:, t] = self._rstate.float().cpu().numpy()
                if explore:
                    a, lp, v, logits, self._rstate = self.module.forward_exploration_step(o, self._rstate)
                else:
                    a, v, self._rstate = self.module.forward_inference_step(o, self._rstate)
                    lp, logits = torch.zeros(N, device=o.device), None
            elif explore:
                a, lp, v, logits = self.module.forward_exploration(o)
            else:
                a, v = self.module.forward_inference(o)
                lp = torch.zeros(N, device=o.device)
                logits = None
            if gpu:
                a, lp, v, logits = self._to_host(a, lp, v, logits)
            if prof is not None:
                t2 = clk()
                prof["inference_s"] = prof.get("inference_s", 0.0) + (t2 - t1)
            if logits is not None:
                if logits_buf is None:
                    logits_buf = np.empty((N, T, logits.shape[-1]), dtype=np.float32)
                logits_buf[:, t] = logits.numpy()
            obs_buf[:, t] = mobs
            an = a.numpy()
            acts[:, t] = an
            logp[:, t] = lp.numpy()
            vf[:, t] = v.numpy()
            if prof is None:
                nobs, r, te, tr, info = self.env.step(self._env_actions(an, explore))
            else:
                t3 = clk()
                ea = self._env_actions(an, explore)
                t4 = clk()
                nobs, r, te, tr, info = self.env.step(ea)
                t5 = clk()
                prof["buffers_s"] = prof.get("buffers_s", 0.0) + (t3 - t2)
                prof["module_to_env_s"] = prof.get("module_to_env_s", 0.0) + (t4 - t3)
                prof["env_step_s"] = prof.get("env_step_s", 0.0) + (t5 - t4)
            rew[:, t] = r
            term[:, t] = te
            trunc[:, t] = tr
            eid_buf[:, t] = self._eps_ids
            for i in np.nonzero(te | tr)[0]:
                self._eps_ids[i] = self._eps_next
                self._eps_next += 1
            if tr.any():
                idx = np.nonzero(tr)[0]
                fo = self._peek_obs(info["final_obs"][idx], idx, an, r)
                trunc_fix.append((t, idx, fo, self._rstate[torch.from_numpy(idx)] if self.stateful else None))
            self._track(r, te, tr, info)
            self.obs = nobs
            ctx.is_first = te | tr
            ctx.last_actions, ctx.last_rewards = an, r
            if prof is not None:
                prof["bookkeeping_s"] = prof.get("bookkeeping_s", 0.0) + (clk() - t5)
        t_loop = clk()
        # bootstrap V(s_T): the next fragment starts from these module inputs (connector state
        # advances exactly once per env step)
        self._pending_mobs = self._module_obs(self.obs, explore)
        st_next = None
        if self.stateful:
            st_next = self._rstate.clone()
            if ctx.is_first.any():
                st_next[torch.from_numpy(ctx.is_first).to(st_next.device)] = 0.0
        last_v = self._value(self._pending_mobs, st_next)
        next_vf = np.empty_like(vf)
        next_vf[:, :-1] = vf[:, 1:]
        next_vf[:, -1] = last_v
        for t, idx, fo, st in trunc_fix:
            next_vf[idx, t] = self._value(fo, st)
        self.steps_sampled += N * T
        b = SampleBatch({SampleBatch.OBS: obs_buf, SampleBatch.ACTIONS: acts, SampleBatch.ACTION_LOGP: logp,
                         SampleBatch.VF_PREDS: vf, SampleBatch.REWARDS: rew, SampleBatch.TERMINATEDS: term,
                         SampleBatch.TRUNCATEDS: trunc, SampleBatch.NEXT_VF_PREDS: next_vf,
                         SampleBatch.EPS_ID: eid_buf})
        if logits_buf is not None:
            b[SampleBatch.ACTION_DIST_INPUTS] = logits_buf
        if self.stateful:
            b["state_in"] = state_buf
            b["is_first"] = first_buf
        b.fragment_shape = (N, T)
        if self.cfg.get("output"):
            if getattr(self, "_writer", None) is None:
                from ..offline import JsonWriter

                self._writer = JsonWriter(self.cfg["output"])
            self._writer.write(b)
        if self.callbacks is not None:
            self.callbacks.on_sample_end(env_runner=self, samples=b)
        if prof is not None:
            end = clk()
            prof["bootstrap_and_assembly_s"] = prof.get("bootstrap_and_assembly_s", 0.0) + (end - t_loop)
            prof["sample_total_s"] = prof.get("sample_total_s", 0.0) + (end - t_start)
            prof["steps"] = prof.get("steps", 0) + N * T
            prof["fragments"] = prof.get("fragments", 0) + 1
        return b

    def sample_profile(self, reset: bool = True) -> Dict:
        """The accumulated per-phase times of ``sample()`` (empty unless ``profile_env_runner``)."""
        out = dict(self._prof or {})
        if reset and self._prof is not None:
            self._prof.clear()
        return out

    @torch.no_grad()
    def sample_transitions(self, num_steps: int, epsilon: float = 0.0) -> SampleBatch:
        """Off-policy transitions (DQN: epsilon-greedy on the Q head; SAC: the stochastic policy
        with probability-epsilon uniform actions). Observations go through the env-to-module
        pipeline exactly as on the on-policy path -- ``obs`` / ``new_obs`` are module inputs (e.g.
        stacked frames, MeanStd-normalised) and connector state advances once per env step; the
        final observation of an ended episode is the pipeline's view of it WITHOUT committing state
        (``_peek_obs``). Actions are stored in module space and sent through module-to-env."""
        N = self.N
        T = max(1, int(num_steps) // N)
        out = {k: [] for k in ("obs", "actions", "rewards", "new_obs", "terminateds")}
        continuous = not hasattr(self.module, "q_values")
        space = self.env.action_space
        conn = len(self.env_to_module) > 0
        ctx = self._ctx
        for _ in range(T):
            if self._pending_mobs is not None:
                mobs, self._pending_mobs = self._pending_mobs, None
            else:
                mobs = self._module_obs(self.obs, True)
            o = torch.from_numpy(np.ascontiguousarray(mobs))
            if continuous:  # SAC: stochastic policy; epsilon = probability of a uniform random action
                a = self.module.forward_exploration(o)[0].numpy().astype(np.float32)
                rnd = self._rng.random(N) < epsilon
                if rnd.any():
                    lo, hi = ((-1.0, 1.0) if self.cfg.get("normalize_actions") else (space.low, space.high))
                    a[rnd] = self._rng.uniform(lo, hi, size=(int(rnd.sum()),) + space.shape)
            else:
                q = self.module.q_values(o)
                a = q.argmax(-1).numpy()
                rnd = self._rng.random(N) < epsilon
                if rnd.any():
                    a[rnd] = self._rng.integers(0, space.n, int(rnd.sum()))
            nobs, r, te, tr, info = self.env.step(self._env_actions(a, True))
            done = te | tr
            if conn:
                nxt = None
                if done.any():  # peek the ended episodes' final observations before state moves on
                    idx = np.nonzero(done)[0]
                    fin = self._peek_obs(info["final_obs"][idx], idx, a, r)
                ctx.is_first = done
                ctx.last_actions, ctx.last_rewards = a, r
                self._pending_mobs = self._module_obs(nobs, True)  # the next step's module input
                nxt = np.array(self._pending_mobs, copy=True)
                if done.any():
                    nxt[idx] = fin
            else:
                nxt = np.where(done.reshape((-1,) + (1,) * (nobs.ndim - 1)), info["final_obs"], nobs)
                ctx.is_first = done
                ctx.last_actions, ctx.last_rewards = a, r
            out["obs"].append(mobs)
            out["actions"].append(a)
            out["rewards"].append(r)
            out["new_obs"].append(nxt)
            out["terminateds"].append(te)
            self._track(r, te, tr, info)
            self.obs = nobs
        self.steps_sampled += N * T
        b = SampleBatch({k: np.concatenate(v, axis=0) if k in ("obs", "new_obs") else np.concatenate(v) for k, v
                         in out.items()})
        if self.callbacks is not None:
            self.callbacks.on_sample_end(env_runner=self, samples=b)
        return b

    # ------------------------------------------------------------------ episodes (new API stack)
    @torch.no_grad()
    def sample_episodes(self, num_timesteps: int, explore: bool = True, epsilon: float = 0.0,
                        frame_stack: int = 1):
        """Sample ``num_timesteps`` env steps as ``SingleAgentEpisode`` chunks (reference:
        ``SingleAgentEnvRunner.sample`` returning episodes). One episode per sub-env is kept
        across calls; the call returns every episode that finished plus the chunk of every
        ongoing one, and continues those with ``cut(frame_stack - 1)`` so the next chunk's
        lookback holds the frames its first stack needs. The module's input is read FROM the
        episodes: the last observation, or with ``frame_stack > 1`` the stack of the last
        ``frame_stack`` observations (zeros before the episode's start) -- an episode-reading
        frame-stacking connector, no per-env history kept anywhere else. Q-modules (DQN) act
        epsilon-greedy; policy modules sample and record ``action_logp`` / ``vf_preds``."""
        from .single_agent_episode import SingleAgentEpisode

        N = self.N
        fs = max(1, int(frame_stack))
        if getattr(self, "_episodes", None) is None or getattr(self, "_episodes_fs", None) != fs:
            self._episodes = []
            for i in range(N):
                ep = SingleAgentEpisode(observation_space=self.env.observation_space,
                                        action_space=self.env.action_space)
                ep.add_env_reset(np.asarray(self.obs[i]))
                self._episodes.append(ep)
            self._episodes_fs = fs
        T = max(1, int(num_timesteps) // N)
        done_eps = []
        q_mode = hasattr(self.module, "q_values")
        space = self.env.action_space
        for _ in range(T):
            if fs > 1:
                mobs = np.stack([ep.get_frame_stack(fs) for ep in self._episodes]).astype(np.float32)
            else:
                mobs = np.stack([np.asarray(ep.get_observations(-1)) for ep in self._episodes]).astype(np.float32)
            o = torch.from_numpy(np.ascontiguousarray(mobs))
            extra = None
            if q_mode:
                a = self.module.q_values(o).argmax(-1).numpy()
                if explore and epsilon > 0:
                    rnd = self._rng.random(N) < epsilon
                    if rnd.any():
                        a[rnd] = self._rng.integers(0, space.n, int(rnd.sum()))
            elif explore:
                at, lp, v, _ = self.module.forward_exploration(o)
                a = at.numpy()
                extra = {"action_logp": lp.numpy(), "vf_preds": v.numpy()}
            else:
                at, v = self.module.forward_inference(o)
                a = at.numpy()
            nobs, r, te, tr, info = self.env.step(a)
            for i, ep in enumerate(self._episodes):
                done = bool(te[i] or tr[i])
                fin = np.asarray(info["final_obs"][i] if done else nobs[i])
                ep.add_env_step(fin, a[i], float(r[i]), terminated=bool(te[i]), truncated=bool(tr[i]) and not te[i],
                                extra_model_outputs=None if extra is None else {k: v[i] for k, v in extra.items()})
                if done:
                    done_eps.append(ep)
                    nxt = SingleAgentEpisode(observation_space=self.env.observation_space,
                                             action_space=self.env.action_space)
                    nxt.add_env_reset(np.asarray(nobs[i]))
                    self._episodes[i] = nxt
            self._track(r, te, tr, info)
            self.obs = nobs
        self.steps_sampled += N * T
        out = [ep.finalize() for ep in done_eps]
        for i, ep in enumerate(self._episodes):
            if len(ep):
                out.append(ep)
                self._episodes[i] = ep.cut(len_lookback_buffer=fs - 1)
        for ep in out:
            ep.finalize()
        return out

    def get_metrics(self) -> Dict:
        eps, cms = self.new_episodes, self.new_custom_metrics
        self.new_episodes, self.new_custom_metrics = [], []
        return {"episodes": eps, "num_env_steps_sampled": self.steps_sampled, "custom_metrics": cms}

    def ping(self):
        return "ok"

    def assert_healthy(self) -> None:
        """Raises if this runner cannot sample (no env, or a module without weights)."""
        assert self.env is not None and getattr(self.env, "num_envs", 0) > 0, "env runner has no env"
        assert self.module is not None, "env runner has no RLModule"

    def stop(self) -> None:
        """Close the sub-environments (envs with a ``close()``)."""
        for e in getattr(self.env, "envs", []) or []:
            close = getattr(e, "close", None)
            if callable(close):
                try:
                    close()
                except Exception:
                    pass

    def apply(self, func, *args, **kwargs):
        """``func(self, *args)`` (``EnvRunnerGroup.foreach_env_runner`` with a callable)."""
        return func(self, *args, **kwargs)


class ExternalInputRunner(EnvRunner):
    """Env runner fed by an input reader instead of an env (reference: a RolloutWorker whose
    ``input_`` is a reader factory, e.g. ``PolicyServerInput``): ``config["input_"]`` is called
    with an ``IOContext`` (config + this runner, whose module answers the reader's action
    requests); ``sample`` returns the reader's next batch. Spaces come from
    ``config.environment(observation_space=..., action_space=...)``."""

    def __init__(self, config: Dict, worker_index: int = 0):
        import threading

        from .policy_server_input import IOContext

        torch.set_num_threads(int(config.get("num_cpus_per_env_runner_threads", 1)))
        self.cfg = config
        self.worker_index = worker_index
        self.observation_space = config.get("observation_space")
        self.action_space = config.get("action_space")
        if self.observation_space is None or self.action_space is None:
            raise ValueError("an external input needs config.environment(observation_space=..., action_space=...)")
        self._module_obs_space = self.observation_space
        self.N = 1
        self.env = None
        self.module = make_module(config, self.observation_space, self.action_space)
        self.module.eval()
        self.stateful = False
        self.device = torch.device("cpu")
        self._module_lock = threading.Lock()
        self.weights_version = -1
        self.steps_sampled = 0
        self.completed = collections.deque(maxlen=int(config.get("metrics_num_episodes_for_smoothing", 100)))
        self.new_episodes = []
        self.new_custom_metrics = []
        self.callbacks = None
        self.env_to_module = self.module_to_env = []
        self.reader = config["input_"](IOContext(config, self, worker_index))

    def spaces(self):
        return self.observation_space, self.action_space

    def set_weights(self, state, version: int = 0):
        with self._module_lock:
            return super().set_weights(state, version)

    def get_connector_state(self):
        return {}

    def set_connector_state(self, state):
        return True

    def sample(self, num_steps: Optional[int] = None, explore: bool = True) -> SampleBatch:
        b = self.reader.next(num_steps)
        self.steps_sampled += b.count
        pop = getattr(self.reader, "pop_episode_returns", None)
        for ret, n in (pop() if pop is not None else []):
            self.completed.append((ret, n))
            self.new_episodes.append((ret, n))
        return b
