"""Train AMP / accelerator tests (reference: train/torch/train_loop_utils.py accelerate,
prepare_optimizer, backward, _TorchAccelerator; train/tests/test_torch_amp.py-style checks)."""
import json
import os
import pickle

import pytest
import torch

from ray_community_amd import train
from ray_community_amd.train import RunConfig, ScalingConfig
from ray_community_amd.train.torch import TorchTrainer


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = torch.nn.Linear(8, 16)
        self.l2 = torch.nn.Linear(16, 1)

    def forward(self, x):
        h = self.l1(x)
        self.seen = (h.dtype, torch.is_autocast_enabled("cpu"))
        return self.l2(torch.relu(h))


def _amp_loop(config):
    from ray_community_amd.train import torch as rt

    rt.accelerate(amp=True, dtype=getattr(torch, config["dtype"]))
    with pytest.raises(RuntimeError, match="already been set"):
        rt.accelerate(amp=True)
    torch.manual_seed(0)
    net = _Net()
    model = rt.prepare_model(net)
    opt = rt.prepare_optimizer(torch.optim.SGD(model.parameters(), lr=0.05))
    x = torch.randn(32, 8)
    y = x.sum(1, keepdim=True)
    losses = []
    for _ in range(5):
        out = model(x)
        loss = torch.nn.functional.mse_loss(out.float(), y)
        rt.backward(loss)
        opt.step()
        opt.zero_grad()
        losses.append(float(loss.detach()))
    inner = model.module if hasattr(model, "module") else model
    train.report({"losses": losses, "act_dtype": str(net.seen[0]), "autocast": net.seen[1],
                  "param_dtype": str(next(inner.parameters()).dtype),
                  "scaler": opt.scaler is not None})


@pytest.mark.parametrize("dtype,scaler", [("bfloat16", False), ("float16", True)])
def test_accelerate_amp_autocast_in_train_loop(ray_start_regular, tmp_path, dtype, scaler):
    t = TorchTrainer(_amp_loop, train_loop_config={"dtype": dtype}, scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(name=f"amp_{dtype}", storage_path=str(tmp_path)))
    m = t.fit().metrics
    assert m["autocast"] is True
    assert m["act_dtype"] == f"torch.{dtype}"     # matmul outputs in the autocast dtype
    assert m["param_dtype"] == "torch.float32"    # fp32 master parameters
    assert m["scaler"] is scaler                   # bf16 needs no loss scaling, fp16 gets a GradScaler
    assert m["losses"][-1] < m["losses"][0]


def test_no_accelerate_is_full_precision():
    from ray_community_amd.train.torch import train_loop_utils as tlu

    tlu._ACCEL.update(explicit=None, default=None)
    net = tlu.prepare_model(_Net())
    net(torch.randn(4, 8))
    assert net.seen == (torch.float32, False)
    opt = tlu.prepare_optimizer(torch.optim.SGD(net.parameters(), lr=0.1))
    assert opt.scaler is None and opt.param_groups[0]["lr"] == 0.1
    loss = net(torch.randn(4, 8)).sum()
    tlu.backward(loss)
    assert net.l1.weight.grad is not None
    opt.step()
    opt.zero_grad()
    assert net.l1.weight.grad is None


def test_amp_model_pickles_with_its_original_forward():
    from ray_community_amd.train.torch import train_loop_utils as tlu

    tlu._ACCEL.update(explicit=None, default=None)
    tlu.accelerate(amp=True)
    try:
        net = tlu.prepare_model(_Net())
        net(torch.randn(2, 8))
        assert net.seen == (torch.bfloat16, True)
        back = pickle.loads(pickle.dumps(net))
        back(torch.randn(2, 8))
        assert back.seen == (torch.float32, False)  # the unwrapped forward travelled
        assert torch.equal(back.l1.weight, net.l1.weight)
    finally:
        tlu._ACCEL.update(explicit=None, default=None)


def test_fp16_scaler_skips_inf_steps():
    """An overflowing fp16 step is skipped by the GradScaler and the scale shrinks."""
    from ray_community_amd.train.torch import train_loop_utils as tlu

    tlu._ACCEL.update(explicit=None, default=None)
    tlu.accelerate(amp=True, dtype=torch.float16)
    try:
        net = tlu.prepare_model(torch.nn.Linear(4, 1))
        opt = tlu.prepare_optimizer(torch.optim.SGD(net.parameters(), lr=0.1))
        w0 = net.weight.detach().clone()
        s0 = opt.scaler.get_scale()
        loss = net(torch.randn(2, 4)).float().sum() * float("inf")
        tlu.backward(loss)
        opt.step()
        assert torch.equal(net.weight.detach(), w0)
        assert opt.scaler.get_scale() < s0
    finally:
        tlu._ACCEL.update(explicit=None, default=None)


def test_torch_worker_profiler_writes_traces(tmp_path):
    from ray_community_amd.train.torch import TorchWorkerProfiler

    prof = TorchWorkerProfiler(trace_dir=str(tmp_path),
                               schedule=torch.profiler.schedule(wait=0, warmup=0, active=2, repeat=1))
    net = torch.nn.Linear(8, 8)
    with prof.profiler as p:
        for _ in range(3):
            net(torch.randn(4, 8)).sum().backward()
            p.step()
    out = prof.get_and_clear_profile_traces()["profiler_traces"]
    assert len(out) == 1
    name, blob = out[0]
    assert name.startswith("worker_0_trace_") and os.path.exists(tmp_path / name)
    trace = json.loads(blob)
    assert any("addmm" in ev.get("name", "") or "linear" in ev.get("name", "") for ev in trace["traceEvents"])
    assert prof.get_and_clear_profile_traces()["profiler_traces"] == []
