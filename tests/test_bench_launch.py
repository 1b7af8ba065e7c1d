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
    assert rec["config"]["launch"] == "torchrun" and rec["config"]["grad_reduce_dtype"] == "fp32"


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
    assert rec["config"]["parallel_mode"] == "ddp" and rec["config"]["launch"] == "TorchTrainer worker actors"
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
