#!/usr/bin/env python3
"""Secondary benchmark: RLlib PPO env-steps/sec on the Atari-shaped task (BASELINE.json config
"RLlib PPO Atari, GPU learners + vectorized env actors (SampleBatch HIP GAE)").

    python bench_rllib.py --learners L --runners R --envs-per-runner E --iters K --warmup W

Env runners are CPU actors stepping E vectorised SyntheticAtari envs (84x84x4 uint8, Discrete(6):
ALE is not installed here); the learner(s) run on MI355X GPUs (GAE / advantage normalisation /
frame preprocessing as HIP kernels; with L > 1 learners, gradients all-reduced over RCCL).
Prints ONE JSON line with whole-job env-steps/s over K timed training iterations.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--learners", type=int, default=None,
                    help="GPU learner actors (default: one per visible GPU; 0 = a local learner in the driver)")
    ap.add_argument("--runners", type=int, default=None)
    ap.add_argument("--envs-per-runner", type=int, default=16)
    ap.add_argument("--train-batch", type=int, default=8192)
    ap.add_argument("--minibatch", type=int, default=1024)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--env", default="ALE/Pong-v5")
    ap.add_argument("--runner-gpu-share", type=float, default=0.0,
                    help="fraction of each GPU given to env-runner policy inference (0: runners infer on CPU); "
                         "the learner on that GPU gets the rest. Measured on 1x MI355X: 0.5 -> 35.1k env-steps/s "
                         "(12 runners x 22 envs: env stepping dominates, the learner slows on half a GPU) vs "
                         "40.9k with 16 CPU-inference runners, so off by default")
    ap.add_argument("--profile-runner", action="store_true",
                    help="per-phase breakdown of the env runners' sample loop (connectors, inference, env step, "
                         "bookkeeping, fragment assembly) and of the driver's iteration, in the JSON's extra")
    args = ap.parse_args()

    import torch

    import ray_community_amd as ray
    from ray_community_amd.rllib import PPOConfig

    ncpu = len(os.sched_getaffinity(0))
    runners = args.runners if args.runners is not None else max(1, min(16, ncpu - 2))
    ngpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if args.learners is None:
        args.learners = ngpu
    ray.init(num_cpus=max(ncpu, runners + 2), num_gpus=ngpu, log_to_driver=False)
    share = args.runner_gpu_share if ngpu else 0.0
    if share > 0 and args.runners is None and runners > 12 * ngpu:
        # GPU-inference runners each open the device: keep <= 12 per GPU (+ learner, driver) and
        # the same total number of vectorised envs
        total_envs = runners * args.envs_per_runner
        runners = 12 * ngpu
        args.envs_per_runner = -(-total_envs // runners)
    # resources are fixed-point 1e-4 units: round the per-runner share DOWN so runners + learner fit
    per_runner = int(share * ngpu / runners * 1e4) / 1e4 if share > 0 else 0
    cfg = (PPOConfig().environment(args.env)
           .env_runners(num_env_runners=runners, num_envs_per_env_runner=args.envs_per_runner,
                        num_gpus_per_env_runner=per_runner)
           .training(lr=2.5e-4, train_batch_size=args.train_batch, minibatch_size=args.minibatch,
                     num_epochs=args.epochs, clip_param=0.1, vf_clip_param=10.0, entropy_coeff=0.01,
                     kl_coeff=0.5, lambda_=0.95, gamma=0.99, model={"vf_share_layers": True}))
    if args.profile_runner:
        cfg.profile_env_runner = True
    if args.learners > 0:
        cfg.learners(num_learners=args.learners, num_gpus_per_learner=(1.0 - share) if ngpu else 0)
    else:
        cfg.resources(num_gpus=1 if ngpu else 0)
    import threading

    t_start = time.perf_counter()
    stop = threading.Event()

    def heartbeat():  # long first-iteration kernel builds (MIOpen) must not look like a hang
        while not stop.wait(30):
            print(f"[bench_rllib] still running ({time.perf_counter() - t_start:.0f} s)", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    algo = cfg.build()
    print(f"[bench_rllib] built in {time.perf_counter() - t_start:.1f} s", file=sys.stderr, flush=True)
    for i in range(args.warmup):
        algo.train()
        print(f"[bench_rllib] warmup {i} done at {time.perf_counter() - t_start:.1f} s", file=sys.stderr, flush=True)
    if args.profile_runner:
        algo.env_runner_group.foreach_env_runner("sample_profile")  # drop the warmup's numbers
    t0 = time.perf_counter()
    steps = 0
    last = None
    phases = {"sample_time_s": 0.0, "learn_time_s": 0.0, "sync_weights_time_s": 0.0}
    for _ in range(args.iters):
        r = algo.train()
        steps += r["num_env_steps_sampled_this_iter"]
        last = r
        li = r["info"]["learner"]["default_policy"]
        for k in phases:
            phases[k] += float(li.get(k, 0.0))
    dt = time.perf_counter() - t0
    runner_profile = None
    if args.profile_runner:
        profs = [p for p in algo.env_runner_group.foreach_env_runner("sample_profile") if p]
        if profs:
            keys = sorted({k for p in profs for k in p if k.endswith("_s")})
            frag = sum(p.get("fragments", 0) for p in profs)
            # mean per fragment over all runners, ms
            runner_profile = {k[:-2] + "_ms_per_fragment": round(1e3 * sum(p.get(k, 0.0) for p in profs)
                                                                        / max(1, frag), 3) for k in keys}
            runner_profile["fragments"] = frag
            runner_profile["steps_per_fragment"] = round(sum(p.get("steps", 0) for p in profs) / max(1, frag), 1)
    out = {"metric": "rllib_ppo_env_steps_per_sec", "value": round(steps / dt, 1), "unit": "env-steps/s",
           "n_gpus": max(1, args.learners) if ngpu else 0, "iters": args.iters, "warmup": args.warmup,
           "higher_is_better": True, "vs_baseline": None, "data": "SyntheticAtari (84x84x4 uint8, Discrete(6))",
           "config": {"env_runners": runners, "envs_per_runner": args.envs_per_runner,
                      "train_batch_size": args.train_batch, "minibatch": args.minibatch, "epochs": args.epochs,
                      "learners": args.learners, "runner_gpu_share": share},
           "extra": {"learner_time_s": last["info"]["learner"]["default_policy"].get("learner_time_s"),
                     "iter_time_s": dt / max(1, args.iters),
                     "driver_phase_s_per_iter": {k: round(v / max(1, args.iters), 4) for k, v in phases.items()},
                     "runner_profile": runner_profile}}
    stop.set()
    print(json.dumps(out), flush=True)
    algo.stop()
    ray.shutdown()


if __name__ == "__main__":
    main()
