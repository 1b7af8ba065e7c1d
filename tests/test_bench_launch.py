"""The driver's multi-GPU launch path of bench.py (torchrun -> TorchTrainer external-launcher mode
-> bucketed DDP), rehearsed on CPU with gloo and the tiny Llama preset."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_torchrun_two_ranks_cpu(tmp_path):
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29541", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--model", "llama3-tiny", "--seq-len", "128", "--device", "cpu", "--parallel", "zero",
           "--grad-reduce-dtype", "fp32"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints exactly one JSON line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["value"] > 0
    assert rec["steps"] == 2 and rec["warmup"] == 1 and rec["higher_is_better"] is True
    assert "ZeRO" in rec["config"]["data_parallel"] and rec["config"]["parallel_mode"] == "zero"
    # a sharded optimizer is not the DDP headline: it reports under its own metric name
    assert rec["metric"] == "ray_train_tokens_per_sec_llama3_8b_zero"
    assert rec["config"]["launch"] == "torchrun" and rec["config"]["grad_reduce_dtype"] == "fp32"
    # per-rank step times: the job's ms/step is the slowest rank's
    ranks = rec["extra"]["rank_ms_per_step"]
    assert len(ranks) == 2 and rec["extra"]["rank_ms_per_step_max"] == max(ranks)
    assert abs(rec["ms_per_step"] - max(ranks)) < 1e-2 and rec["extra"]["rank_ms_per_step_min"] == min(ranks)


def test_bench_self_launch_two_workers_cpu(tmp_path):
    """``bench.py --gpus 2`` without torchrun: TorchTrainer starts two Train worker actors that
    form a (gloo, on CPU) process group; n_gpus comes from the group's world size."""
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--model", "llama3-tiny", "--seq-len", "128", "--device", "cpu"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["value"] > 0
    # the default --parallel is ddp at every N, matching the headline metric's name
    assert rec["config"]["parallel_mode"] == "ddp" and rec["config"]["launch"] == "TorchTrainer worker actors"
    assert rec["metric"] == "ray_train_tokens_per_sec_llama3_8b_ddp"
    assert rec["extra"]["exposed_comm_ms"] == 0.0  # events are only recorded on GPUs
    assert rec["config"]["global_batch"] == 4


def test_bench_data_serve_pipeline_cpu(tmp_path):
    """Config 5 plumbing: Data read -> map_batches actor pool -> Serve handle -> replica, on CPU."""
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench_data_serve.py"), "--device", "cpu", "--model", "tiny",
           "--image-size", "32", "--batch-size", "16", "--batches", "4", "--warmup", "2"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and rec["steps"] == 4 and rec["extra"]["images"] == 6 * 16


def test_bench_data_serve_eight_replicas_cpu(tmp_path):
    """The 8-GPU config-5 shape rehearsed on CPU: 8 Serve replicas behind the router, 16
    preprocess actors; per-replica load/latency and the hand-off time are reported."""
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench_data_serve.py"), "--gpus", "8", "--device", "cpu", "--model",
           "tiny", "--image-size", "32", "--batch-size", "16", "--batches", "24", "--warmup", "4"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["config"]["replicas"] == 8 and rec["config"]["preprocess_actors"] == 16
    ex = rec["extra"]
    assert ex["images"] == 28 * 16 and rec["value"] > 0
    assert ex["replicas_used"] >= 4, ex  # power-of-two-choices spreads the 16 callers
    assert sum(r["requests"] for r in ex["per_replica"]) == 24
    assert all(r["rtt_ms"] >= r["infer_ms"] for r in ex["per_replica"]) and ex["handoff_ms_mean"] >= 0


def test_eight_virtual_gpu_workers_get_distinct_devices():
    """8 GPU worker actors on a node with 8 (virtual) GPUs: each sees its own GPU id, the plan
    gives every worker the union 0..7 in HIP_VISIBLE_DEVICES and a distinct device index that
    points back at its own GPU (what _setup_torch_process_group then asserts on real hardware)."""
    import ray_community_amd as ray
    from ray_community_amd.train._internal.worker_group import WorkerGroup
    from ray_community_amd.train.backend import _assign_ranks, _node_info_fn
    from ray_community_amd.train.torch.config import plan_devices

    ray.init(num_cpus=8, num_gpus=8, include_dashboard=False, log_to_driver=False)
    try:
        wg = WorkerGroup(8, {"CPU": 0.5, "GPU": 1})
        infos = _assign_ranks(wg.execute(_node_info_fn))
        plan = plan_devices(infos, use_gpu=True)
        own = [inf["visible"][0] for inf in infos]
        assert sorted(own, key=int) == [str(i) for i in range(8)]
        for inf, (dev, vis) in zip(infos, plan):
            assert vis == [str(i) for i in range(8)]
            assert vis[dev] == inf["visible"][0]
        assert sorted(d for d, _ in plan) == list(range(8))
        assert [inf["local_rank"] for inf in infos] == list(range(8)) and {inf["local_world_size"] for inf in infos} == {8}
        wg.shutdown()
    finally:
        ray.shutdown()


def test_plan_devices_rejects_two_workers_on_one_gpu():
    import pytest as _pt

    from ray_community_amd.train.torch.config import plan_devices

    infos = [{"node_id": "n", "visible": ["3"]}, {"node_id": "n", "visible": ["3"]}]
    with _pt.raises(RuntimeError, match="both use GPU 3"):
        plan_devices(infos, use_gpu=True)
    assert plan_devices(infos, use_gpu=False) == [(None, None), (None, None)]
