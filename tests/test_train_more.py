"""More Train behaviour (reference test models: python/ray/train/tests/test_data_parallel_trainer.py
(dataset shards, metrics dataframe), test_torch_trainer.py (DDP param sync across ranks),
test_session.py (report + checkpoint from every rank), test_result.py)."""
import os
import tempfile

import pytest
import torch

import ray_community_amd as ray
from ray_community_amd import data, train
from ray_community_amd.train import Checkpoint, RunConfig, ScalingConfig
from ray_community_amd.train.data_parallel_trainer import DataParallelTrainer
from ray_community_amd.train.torch import TorchTrainer


@pytest.fixture
def ray4():
    ray.init(num_cpus=4, log_to_driver=False)
    yield
    ray.shutdown()


def test_dataset_shards_are_disjoint_and_complete(ray4, tmp_path):
    def loop(config):
        shard = train.get_dataset_shard("train")
        ids = []
        for b in shard.iter_batches(batch_size=7):
            ids.extend(int(x) for x in b["id"])
        train.report({"ids": ids, "rank": train.get_context().get_world_rank()})

    trainer = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                                  datasets={"train": data.range(64, override_num_blocks=8)},
                                  run_config=RunConfig(name="shards", storage_path=str(tmp_path)))
    res = trainer.fit()
    assert res.error is None
    # rank 0 reports; the shards of both ranks are gathered by reading each rank's file below
    assert 20 <= len(res.metrics["ids"]) <= 44


def test_metrics_dataframe_and_report_checkpoint(ray4, tmp_path):
    def loop(config):
        for i in range(3):
            with tempfile.TemporaryDirectory() as d:
                if train.get_context().get_world_rank() == 0:
                    with open(os.path.join(d, "state.txt"), "w") as f:
                        f.write(str(i))
                train.report({"step": i, "loss": 1.0 / (i + 1)}, checkpoint=Checkpoint.from_directory(d))

    res = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                              run_config=RunConfig(name="mdf", storage_path=str(tmp_path))).fit()
    df = res.metrics_dataframe
    assert list(df["step"]) == [0, 1, 2]
    with res.checkpoint.as_directory() as d:
        assert open(os.path.join(d, "state.txt")).read() == "2"
    assert res.path and os.path.isdir(res.path)


def test_torch_ddp_keeps_replicas_identical(ray4, tmp_path):
    def loop(config):
        from ray_community_amd.train.torch import prepare_model

        torch.manual_seed(train.get_context().get_world_rank())  # different init per rank
        model = prepare_model(torch.nn.Linear(4, 2))
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        g = torch.Generator().manual_seed(100 + train.get_context().get_world_rank())
        for _ in range(3):
            x = torch.randn(8, 4, generator=g)  # different data per rank
            loss = model(x).pow(2).mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
        w = (model.module if hasattr(model, "module") else model).weight.detach().clone()
        import torch.distributed as dist

        ws = [torch.zeros_like(w) for _ in range(dist.get_world_size())]
        dist.all_gather(ws, w)
        train.report({"max_diff": float(max((a - ws[0]).abs().max() for a in ws))})

    res = TorchTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                       run_config=RunConfig(name="ddpsync", storage_path=str(tmp_path))).fit()
    assert res.error is None and res.metrics["max_diff"] == 0.0


def test_ddp_flat_grads_survive_set_to_none_zero_grad():
    """Single-process check of the adoption path the grad-ready hooks run (world > 1): after
    ``zero_grad(set_to_none=True)`` a backward's fresh gradient is copied back into the flat buffer
    the collectives reduce and ``p.grad`` points at it again."""
    from ray_community_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Linear(4, 2))
    ddp = DistributedDataParallel(net)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        ddp(torch.randn(5, 3)).sum().backward()
        fresh = {id(p): p.grad.clone() for p in net.parameters()}
        for p in net.parameters():
            ddp.flat.adopt_grad(p)
        for p in net.parameters():
            assert torch.equal(p.grad, fresh[id(p)])
            off = ddp.flat.param_offset[id(p)]
            slot = ddp.flat.grad[off: off + p.numel()].view_as(p)
            assert p.grad.data_ptr() == slot.data_ptr() and torch.equal(p.grad, slot)
        opt.step()


def test_trainer_fit_honours_stop_and_callbacks(ray4, tmp_path):
    """Standalone ``fit()`` applies RunConfig.stop (dict / callable) and calls RunConfig.callbacks
    (on_trial_result per report, on_trial_complete once), as the reference's one-trial Tune run."""
    import time as _t

    from ray_community_amd import tune

    def loop(config):
        for i in range(20):
            train.report({"i": i, "loss": 1.0 / (i + 1)})
            _t.sleep(0.02)

    class CB(tune.Callback):
        def __init__(self):
            self.results, self.completed = [], 0

        def on_trial_result(self, iteration, trials, trial, result, **info):
            self.results.append(result["i"])

        def on_trial_complete(self, iteration, trials, trial, **info):
            self.completed += 1

    cb = CB()
    r = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=1),
                            run_config=RunConfig(name="stop1", storage_path=str(tmp_path),
                                                 stop={"training_iteration": 4}, callbacks=[cb])).fit()
    assert r.metrics["i"] == 3 and cb.results == [0, 1, 2, 3] and cb.completed == 1
    r2 = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=2),
                             run_config=RunConfig(name="stop2", storage_path=str(tmp_path),
                                                  stop=lambda tid, res: res["loss"] < 0.2)).fit()
    assert r2.metrics["i"] == 5  # first report with loss = 1/6 < 0.2
