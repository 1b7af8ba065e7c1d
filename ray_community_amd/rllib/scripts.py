"""The ``rllib`` command line (reference: ``rllib/scripts.py``, ``rllib/train.py``,
``rllib/evaluate.py``, ``rllib/common.py``).

    python -m ray_community_amd.rllib train --algo PPO --env CartPole-v1 [--config JSON] [--stop JSON]
        [--experiment-name N] [--num-samples K] [--checkpoint-freq F] [--checkpoint-at-end]
        [--storage-path DIR] [--restore CKPT] [--resources-per-trial JSON] [--keep-checkpoints-num K]
        [--checkpoint-score-attr A] [--scheduler fifo] [--scheduler-config JSON] [--resume]
        [--ray-address A] [--ray-num-cpus N] [--ray-num-gpus N] [--ray-object-store-memory B] [-v | --vv]
    python -m ray_community_amd.rllib train file EXPERIMENT.yaml|EXPERIMENT.py [--env E] [--stop JSON] ...
    python -m ray_community_amd.rllib evaluate CHECKPOINT [--algo PPO] [--env E] [--episodes N] [--steps N]
        [--config JSON] [--out FILE [--use-shelve] [--save-info] [--track-progress]]
    python -m ray_community_amd.rllib example list [--filter S] | get ID | run ID

``train`` runs the experiment(s) through ``tune.run`` (one trial per sample, every trial an
Algorithm actor) and prints each trial's last checkpoint with the ``evaluate`` command for it.
An experiment file is the reference's format: YAML ``{name: {run, env, stop, config}}`` (old-stack
config keys such as ``num_workers`` / ``num_sgd_iter`` are accepted), or a Python file defining
``config`` (an ``AlgorithmConfig``) and optionally ``stop``.

``evaluate`` rebuilds the Algorithm from the checkpoint (its ``rllib_checkpoint.json`` names the
algorithm, so ``--algo`` is optional), then rolls the greedy policy out on one environment with
``compute_single_action`` (recurrent modules carry their state across steps) until ``--episodes``
or ``--steps`` is reached, printing each episode's return. ``--out`` keeps the transitions
``[obs, action, next_obs, reward, terminated, truncated(, info)]`` per episode: one pickle of the
list of episodes, or a ``shelve`` database keyed by episode index plus ``"num_episodes"``.
Multi-agent checkpoints are evaluated through ``Algorithm.evaluate()`` rounds.
"""
from __future__ import annotations

import argparse
import json
import os
import pickle
import shelve
import sys
import uuid
from pathlib import Path
from typing import Dict, List, Optional

# Built-in examples (reference ``rllib/common.py`` EXAMPLES, which point at tuned_examples files):
# each is an experiment spec, runnable here without downloading anything.
EXAMPLES: Dict[str, Dict] = {
    "cartpole-ppo": {"description": "PPO on CartPole-v1 (reaches return 150 in a few iterations)",
                     "run": "PPO", "env": "CartPole-v1",
                     "stop": {"env_runners/episode_return_mean": 150, "timesteps_total": 100000},
                     "config": {"gamma": 0.99, "lr": 0.0003, "num_env_runners": 1, "num_epochs": 6,
                                "vf_loss_coeff": 0.01}},
    "cartpole-dqn": {"description": "DQN on CartPole-v1", "run": "DQN", "env": "CartPole-v1",
                     "stop": {"env_runners/episode_return_mean": 150, "timesteps_total": 100000},
                     "config": {"num_env_runners": 0}},
    "cartpole-impala": {"description": "IMPALA on CartPole-v1", "run": "IMPALA", "env": "CartPole-v1",
                        "stop": {"env_runners/episode_return_mean": 150, "timesteps_total": 500000},
                        "config": {"num_env_runners": 2}},
    "cartpole-appo": {"description": "APPO on CartPole-v1", "run": "APPO", "env": "CartPole-v1",
                      "stop": {"env_runners/episode_return_mean": 150, "timesteps_total": 500000},
                      "config": {"num_env_runners": 2}},
    "pendulum-sac": {"description": "SAC on Pendulum-v1", "run": "SAC", "env": "Pendulum-v1",
                     "stop": {"env_runners/episode_return_mean": -250, "timesteps_total": 20000},
                     "config": {"num_env_runners": 0}},
    "pendulum-ppo": {"description": "PPO on Pendulum-v1", "run": "PPO", "env": "Pendulum-v1",
                     "stop": {"env_runners/episode_return_mean": -400, "timesteps_total": 400000},
                     "config": {"num_env_runners": 2, "lambda": 0.1, "gamma": 0.95, "lr": 0.0003,
                                "train_batch_size": 4000, "num_epochs": 6}},
    "atari-ppo": {"description": "PPO on the synthetic Atari env (84x84x4 frames, CNN module)",
                  "run": "PPO", "env": "SyntheticAtari-v0",
                  "stop": {"timesteps_total": 5000000},
                  "config": {"num_env_runners": 4, "num_envs_per_env_runner": 8, "train_batch_size": 4096,
                             "minibatch_size": 512, "num_epochs": 2}},
}


# ---------------------------------------------------------------------------------------- train
def load_experiments_from_file(config_file: str, stop: Optional[str] = None,
                               checkpoint_config: Optional[dict] = None) -> Dict[str, Dict]:
    """Experiments dict ``{name: {run, env, stop, config, checkpoint_config}}`` from a YAML file or
    a Python file defining ``config`` (an AlgorithmConfig) and optionally ``stop``."""
    if config_file.endswith((".yaml", ".yml")):
        import yaml

        with open(config_file) as f:
            experiments = yaml.safe_load(f)
        if stop not in (None, "{}"):
            raise ValueError("--stop is only supported with Python experiment files (YAML files carry `stop`)")
    elif config_file.endswith(".py"):
        import importlib.util

        name = Path(config_file).stem
        spec = importlib.util.spec_from_file_location(name, config_file)
        module = importlib.util.module_from_spec(spec)
        sys.modules[name] = module
        spec.loader.exec_module(module)
        if not hasattr(module, "config"):
            raise ValueError("A Python experiment file must define `config` (an AlgorithmConfig)")
        algo_config = module.config
        stop_d = json.loads(stop) if stop is not None else getattr(module, "stop", {})
        cfg = algo_config.to_dict()
        experiments = {f"default_{uuid.uuid4().hex[:8]}": {"run": algo_config.algo_class, "env": cfg.get("env"),
                                                          "config": cfg, "stop": stop_d}}
    else:
        raise ValueError(f"Unsupported experiment file {config_file!r}: use .yaml/.yml or .py")
    if not isinstance(experiments, dict) or not experiments:
        raise ValueError(f"{config_file}: expected a mapping of experiment name -> spec")
    for spec in experiments.values():
        spec["checkpoint_config"] = dict(checkpoint_config or {})
    return experiments


def _ckpt_kwargs(spec: Dict) -> Dict:
    cc = spec.get("checkpoint_config") or {}
    out = {"checkpoint_freq": int(cc.get("checkpoint_frequency") or 0),
           "checkpoint_at_end": bool(cc.get("checkpoint_at_end"))}
    if cc.get("num_to_keep"):
        out["keep_checkpoints_num"] = int(cc["num_to_keep"])
    if cc.get("checkpoint_score_attribute"):
        out["checkpoint_score_attr"] = cc["checkpoint_score_attribute"]
    return out


def run_rllib_experiments(experiments: Dict[str, Dict], *, verbose: int = 1, framework: Optional[str] = None,
                          ray_address: Optional[str] = None, ray_num_cpus: Optional[int] = None,
                          ray_num_gpus: Optional[int] = None, ray_object_store_memory: Optional[int] = None,
                          local_mode: bool = False, resume: bool = False, scheduler: str = "fifo",
                          scheduler_config: str = "{}", algo: Optional[str] = None, callbacks=None,
                          log_level: Optional[str] = None) -> List:
    """Run every experiment through ``tune.run``; returns the trials (reference
    ``rllib/train.py::_run_rllib_experiments``)."""
    import ray_community_amd as ray
    from .. import tune
    from ..tune.registry import create_scheduler

    for spec in experiments.values():
        cfg = spec.setdefault("config", {}) or {}
        spec["config"] = cfg
        if spec.get("env") is not None:
            cfg["env"] = spec["env"]  # a top-level / --env value wins over config.env
        if not cfg.get("env"):
            raise ValueError("Pass --env (e.g. CartPole-v1) or an `env` key in the experiment's config")
        if framework not in (None, "torch"):
            raise ValueError(f"framework {framework!r} is not available: this framework trains with torch on ROCm")
        if log_level:
            cfg["log_level"] = log_level
    owns = not ray.is_initialized()
    if owns:
        kw = {k: v for k, v in (("address", ray_address), ("num_cpus", ray_num_cpus), ("num_gpus", ray_num_gpus),
                                ("object_store_memory", ray_object_store_memory)) if v is not None}
        ray.init(local_mode=local_mode, **kw)
    sched = create_scheduler(scheduler.lower(), **json.loads(scheduler_config or "{}"))
    trials = []
    try:
        for name, spec in experiments.items():
            ana = tune.run(spec.get("run") or algo, name=name, stop=spec.get("stop") or None, config=spec["config"],
                           num_samples=int(spec.get("num_samples") or 1), storage_path=spec.get("storage_path"),
                           resources_per_trial=spec.get("resources_per_trial"), restore=spec.get("restore"),
                           scheduler=sched, resume=resume or None, verbose=verbose, callbacks=callbacks,
                           **_ckpt_kwargs(spec))
            trials.extend(ana.trials)
    finally:
        if owns:
            ray.shutdown()
    ckpts = [t.checkpoint.path for t in trials if getattr(t, "checkpoint", None) is not None]
    if ckpts:
        print("\nYour training finished.\nBest available checkpoint for each trial:")
        for c in ckpts:
            print(f"  {c}")
        run = algo or next(iter(experiments.values())).get("run")
        run = run if isinstance(run, str) else getattr(run, "__name__", str(run))
        print("\nEvaluate a trained algorithm from any checkpoint, e.g.:\n"
              f"  python -m ray_community_amd.rllib evaluate {ckpts[0]} --algo {run}")
    return trials


def _train(args) -> int:
    ckpt = {"checkpoint_frequency": args.checkpoint_freq, "checkpoint_at_end": args.checkpoint_at_end,
            "num_to_keep": args.keep_checkpoints_num, "checkpoint_score_attribute": args.checkpoint_score_attr}
    if getattr(args, "config_file", None):
        experiments = load_experiments_from_file(args.config_file, args.stop, ckpt)
        if args.env is not None:
            for spec in experiments.values():
                spec["env"] = args.env
        for spec in experiments.values():
            spec.setdefault("storage_path", args.storage_path)
        algo = next(iter(experiments.values())).get("run")
    else:
        if not args.algo:
            raise SystemExit("rllib train: --algo is required (or use `rllib train file <file>`)")
        experiments = {args.experiment_name: {
            "run": args.algo, "checkpoint_config": ckpt, "storage_path": args.storage_path,
            "resources_per_trial": json.loads(args.resources_per_trial) if args.resources_per_trial else None,
            "stop": json.loads(args.stop or "{}"), "config": dict(json.loads(args.config or "{}")),
            "env": args.env, "restore": args.restore, "num_samples": args.num_samples}}
        algo = args.algo
    level = "DEBUG" if args.vv else ("INFO" if args.v else None)
    run_rllib_experiments(experiments, verbose=3 if level else 1, framework=args.framework,
                          ray_address=args.ray_address, ray_num_cpus=args.ray_num_cpus,
                          ray_num_gpus=args.ray_num_gpus, ray_object_store_memory=args.ray_object_store_memory,
                          local_mode=args.local_mode, resume=args.resume, scheduler=args.scheduler,
                          scheduler_config=args.scheduler_config, algo=algo if isinstance(algo, str) else None,
                          log_level=level)
    return 0


# ---------------------------------------------------------------------------------------- evaluate
class RolloutSaver:
    """Collects evaluated episodes into ``outfile`` (reference ``rllib/evaluate.py::RolloutSaver``):
    one pickle of ``[episode, ...]`` at the end, or, with ``use_shelve``, a shelve database written
    episode by episode (keys ``"0"``, ``"1"``, ... and ``"num_episodes"``). ``write_update_file``
    keeps a ``__progress_<out>`` file with the progress while the rollout runs."""

    def __init__(self, outfile=None, use_shelve=False, write_update_file=False, target_steps=None,
                 target_episodes=None, save_info=False):
        self.outfile = outfile
        self._use_shelve = use_shelve
        self._write_update = write_update_file
        self._target_steps, self._target_episodes = target_steps, target_episodes
        self._save_info = save_info
        self._shelf = None
        self._update = None
        self._rollouts: List[list] = []
        self._current: list = []
        self.num_episodes = 0
        self.total_steps = 0

    def _progress_path(self) -> Path:
        p = Path(self.outfile)
        return p.parent / ("__progress_" + p.name)

    def __enter__(self):
        if self.outfile:
            if self._use_shelve:
                self._shelf = shelve.open(self.outfile)
            else:
                with open(self.outfile, "wb"):
                    pass  # fail before rolling out if the file cannot be written
            if self._write_update:
                self._update = self._progress_path().open("w")
        return self

    def __exit__(self, *exc):
        if self._shelf is not None:
            self._shelf["num_episodes"] = self.num_episodes
            self._shelf.close()
        elif self.outfile:
            with open(self.outfile, "wb") as f:
                pickle.dump(self._rollouts, f)
        if self._update is not None:
            self._update.close()
            self._progress_path().unlink()
            self._update = None

    def progress(self) -> str:
        if self._target_episodes:
            return f"{self.num_episodes} / {self._target_episodes} episodes completed"
        if self._target_steps:
            return f"{self.total_steps} / {self._target_steps} steps completed"
        return f"{self.num_episodes} episodes completed"

    def begin_rollout(self):
        self._current = []

    def end_rollout(self):
        if self._shelf is not None:
            self._shelf[str(self.num_episodes)] = self._current
        elif self.outfile:
            self._rollouts.append(self._current)
        self.num_episodes += 1
        if self._update is not None:
            self._update.seek(0)
            self._update.write(self.progress() + "\n")
            self._update.flush()

    def append_step(self, obs, action, next_obs, reward, terminated, truncated, info):
        if self.outfile:
            step = [obs, action, next_obs, reward, terminated, truncated]
            if self._save_info:
                step.append(info)
            self._current.append(step)
        self.total_steps += 1


def keep_going(steps: int, num_steps: int, episodes: int, num_episodes: int) -> bool:
    return not ((num_episodes and episodes >= num_episodes) or (num_steps and steps >= num_steps))


def rollout(algo, env_name=None, num_steps: int = 0, num_episodes: int = 0, saver: Optional[RolloutSaver] = None,
            explore: bool = False) -> List[float]:
    """Greedy rollouts of ``algo`` on one environment; returns each finished episode's return."""
    import numpy as np

    from .env.envs import make_vector_env

    saver = saver or RolloutSaver()
    returns: List[float] = []
    if getattr(algo, "multi_agent", False):
        steps = episodes = 0
        while keep_going(steps, num_steps, episodes, num_episodes):
            saver.begin_rollout()
            res = algo.evaluate()
            n = int(res.get("num_episodes") or algo.config.evaluation_duration or 1)
            episodes += n
            steps += n  # per-step counts are not reported by evaluate(); count episodes
            returns.append(float(res["episode_reward_mean"]))
            print(f"Episode #{episodes}: reward: {res['episode_reward_mean']}")
            saver.end_rollout()
        return returns
    cfg = algo.config
    env = make_vector_env(env_name or cfg.env, 1, cfg.env_config, seed=(cfg.seed or 0) + 7)
    module = algo.get_module()
    stateful = bool(getattr(module, "is_stateful", False))
    steps = episodes = 0
    obs, _ = env.reset(seed=(cfg.seed or 0) + 7)
    while keep_going(steps, num_steps, episodes, num_episodes):
        saver.begin_rollout()
        state = None
        total, done = 0.0, False
        while not done and keep_going(steps, num_steps, episodes, num_episodes):
            o = obs[0]
            if stateful:
                a, state, _ = algo.compute_single_action(o, state=state, explore=explore)
            else:
                a = algo.compute_single_action(o, explore=explore)
            nxt, rew, term, trunc, info = env.step(np.asarray([a]))
            te, tr = bool(term[0]), bool(trunc[0])
            done = te or tr
            final = info["final_obs"][0] if done and "final_obs" in info else nxt[0]
            saver.append_step(o, a, final, float(rew[0]), te, tr, {k: v for k, v in info.items() if k != "final_obs"})
            total += float(rew[0])
            steps += 1
            obs = nxt
        saver.end_rollout()
        print(f"Episode #{episodes}: reward: {total}")
        if done:
            episodes += 1
            returns.append(total)
    return returns


def _checkpoint_algo_name(path: str) -> Optional[str]:
    meta = os.path.join(path, "rllib_checkpoint.json")
    if os.path.exists(meta):
        with open(meta) as f:
            return json.load(f).get("algo")
    return None


def evaluate_checkpoint(checkpoint: str, algo: Optional[str] = None, env: Optional[str] = None, steps: int = 0,
                        episodes: int = 0, out: Optional[str] = None, config: str = "{}", save_info: bool = False,
                        use_shelve: bool = False, track_progress: bool = False, local_mode: bool = False,
                        explore: bool = False) -> List[float]:
    import ray_community_amd as ray
    from .algorithms import get_algorithm_class

    if (use_shelve or track_progress) and not out:
        raise ValueError("--use-shelve / --track-progress need an output file (--out)")
    if not steps and not episodes:
        episodes = 1
    ckpt = checkpoint if os.path.isdir(checkpoint) else str(Path(checkpoint).parent)
    name = algo or _checkpoint_algo_name(ckpt)
    if not name:
        raise ValueError(f"{ckpt} does not name its algorithm: pass --algo")
    cls = get_algorithm_class(name)
    if isinstance(cls, tuple):
        cls = cls[0]
    with open(os.path.join(ckpt, "algorithm_state.pkl"), "rb") as f:
        stored = pickle.load(f)["config"]  # written by this framework's Algorithm.save_checkpoint
    overrides = json.loads(config or "{}")
    stored.update(overrides.get("evaluation_config") or stored.get("evaluation_config") or {})
    stored.update(overrides)
    if env:
        stored["env"] = env
    stored["num_env_runners"] = 0  # the rollout runs in this process
    owns = not ray.is_initialized()
    if owns:
        ray.init(local_mode=local_mode)
    try:
        inst = cls(config=cls._default_config_cls().update_from_dict(stored))
        print(f"Restoring algorithm from {ckpt}")
        inst.load_checkpoint(ckpt)
        try:
            with RolloutSaver(out, use_shelve, track_progress, steps, episodes, save_info) as saver:
                return rollout(inst, env, steps, episodes, saver, explore=explore)
        finally:
            inst.stop()
    finally:
        if owns:
            ray.shutdown()


def _evaluate(args) -> int:
    evaluate_checkpoint(args.checkpoint, algo=args.algo, env=args.env, steps=args.steps, episodes=args.episodes,
                        out=args.out, config=args.config, save_info=args.save_info, use_shelve=args.use_shelve,
                        track_progress=args.track_progress, local_mode=args.local_mode, explore=args.explore)
    return 0


# ---------------------------------------------------------------------------------------- examples
def _example(args) -> int:
    if args.example_cmd == "list":
        rows = sorted((k, v["description"]) for k, v in EXAMPLES.items()
                      if not args.filter or args.filter.lower() in k)
        w = max([len(k) for k, _ in rows] + [10])
        print(f"{'Example ID':<{w}}  Description")
        for k, d in rows:
            print(f"{k:<{w}}  {d}")
        print("Run one with `python -m ray_community_amd.rllib example run <Example ID>`.")
        return 0
    if args.example_id not in EXAMPLES:
        raise SystemExit(f"Example {args.example_id} not found; see `example list`")
    spec = {k: v for k, v in EXAMPLES[args.example_id].items() if k != "description"}
    if args.example_cmd == "get":
        import yaml

        print(yaml.safe_dump({args.example_id: spec}, sort_keys=False))
        return 0
    if args.stop:
        spec["stop"] = json.loads(args.stop)
    spec["checkpoint_config"] = {"checkpoint_frequency": 1, "checkpoint_at_end": True,
                                 "checkpoint_score_attribute": "training_iteration"}
    spec["storage_path"] = args.storage_path
    run_rllib_experiments({args.example_id: spec}, verbose=3, algo=spec["run"])
    return 0


# ---------------------------------------------------------------------------------------- parser
def _add_train_common(p: argparse.ArgumentParser):
    p.add_argument("--env", default=None, help="environment name (registered or built in)")
    p.add_argument("--stop", default=None, help="stop criteria as JSON, e.g. '{\"training_iteration\": 10}'")
    p.add_argument("--checkpoint-freq", type=int, default=0)
    p.add_argument("--checkpoint-at-end", action="store_true")
    p.add_argument("--keep-checkpoints-num", type=int, default=None)
    p.add_argument("--checkpoint-score-attr", default="training_iteration")
    p.add_argument("--storage-path", default=None)
    p.add_argument("-v", action="store_true", help="INFO log level, detailed trial results")
    p.add_argument("--vv", action="store_true", help="DEBUG log level")
    p.add_argument("--framework", default=None, choices=["torch"], help="only torch exists here")
    p.add_argument("--local-mode", action="store_true")
    p.add_argument("--ray-address", default=None)
    p.add_argument("--ray-num-cpus", type=int, default=None)
    p.add_argument("--ray-num-gpus", type=int, default=None)
    p.add_argument("--ray-object-store-memory", type=int, default=None)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--scheduler", default="fifo")
    p.add_argument("--scheduler-config", default="{}")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="rllib", description="RLlib command-line interface")
    sub = ap.add_subparsers(dest="cmd", required=True)

    tr = sub.add_parser("train", help="train an algorithm (options) or `train file <experiment file>`")
    _add_train_common(tr)
    tr.add_argument("--algo", "--run", dest="algo", default=None)
    tr.add_argument("--config", default="{}", help="algorithm config overrides as JSON")
    tr.add_argument("--experiment-name", default="default")
    tr.add_argument("--num-samples", type=int, default=1)
    tr.add_argument("--restore", default=None, help="checkpoint directory every trial starts from")
    tr.add_argument("--resources-per-trial", default=None, help="JSON, e.g. '{\"cpu\": 1, \"gpu\": 1}'")
    tsub = tr.add_subparsers(dest="train_cmd")
    tf = tsub.add_parser("file", help="run the experiment(s) in a YAML or Python file")
    tf.add_argument("config_file")
    _add_train_common(tf)

    ev = sub.add_parser("evaluate", help="roll out a trained checkpoint")
    ev.add_argument("checkpoint")
    ev.add_argument("--algo", "--run", dest="algo", default=None)
    ev.add_argument("--env", default=None)
    ev.add_argument("--steps", type=int, default=0)
    ev.add_argument("--episodes", type=int, default=0)
    ev.add_argument("--out", default=None)
    ev.add_argument("--config", default="{}")
    ev.add_argument("--save-info", action="store_true")
    ev.add_argument("--use-shelve", action="store_true")
    ev.add_argument("--track-progress", action="store_true")
    ev.add_argument("--local-mode", action="store_true")
    ev.add_argument("--explore", action="store_true", help="sample actions instead of the greedy policy")
    ev.add_argument("--render", action="store_true", help="accepted for compatibility; the envs here do not render")

    ex = sub.add_parser("example", help="list / show / run the built-in examples")
    esub = ex.add_subparsers(dest="example_cmd", required=True)
    el = esub.add_parser("list")
    el.add_argument("--filter", "-f", default=None)
    eg = esub.add_parser("get")
    eg.add_argument("example_id")
    er = esub.add_parser("run")
    er.add_argument("example_id")
    er.add_argument("--stop", default=None, help="override the example's stop criteria (JSON)")
    er.add_argument("--storage-path", default=None)
    return ap


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    if args.cmd == "train":
        if getattr(args, "train_cmd", None) != "file":
            args.config_file = None
        return _train(args)
    if args.cmd == "evaluate":
        return _evaluate(args)
    return _example(args)


if __name__ == "__main__":
    sys.exit(main())
