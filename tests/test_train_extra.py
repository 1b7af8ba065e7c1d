"""More Ray Train behaviour (reference train/tests/test_checkpoint_manager.py,
test_torch_trainer.py, test_session.py, test_result.py): top-k checkpoint retention by score,
the worker context, DistributedSampler sharding through prepare_data_loader, metrics history,
restore from a run directory."""
import json
import os
import tempfile

import pytest
import torch

import ray_community_amd as ray
from ray_community_amd import train
from ray_community_amd.train import Checkpoint, CheckpointConfig, RunConfig, ScalingConfig
from ray_community_amd.train.torch import TorchTrainer


def _scored_loop(config):
    for epoch in range(config["epochs"]):
        acc = [0.1, 0.9, 0.4, 0.8, 0.2][epoch]
        with tempfile.TemporaryDirectory() as d:
            with open(os.path.join(d, "state.json"), "w") as f:
                json.dump({"epoch": epoch}, f)
            ck = Checkpoint.from_directory(d) if train.get_context().get_world_rank() == 0 else None
            train.report({"epoch": epoch, "acc": acc}, checkpoint=ck)


def test_checkpoint_top_k_by_score(ray_start_regular, tmp_path):
    trainer = TorchTrainer(_scored_loop, train_loop_config={"epochs": 5},
                           scaling_config=ScalingConfig(num_workers=2),
                           run_config=RunConfig(name="topk", storage_path=str(tmp_path),
                                                checkpoint_config=CheckpointConfig(
                                                    num_to_keep=2, checkpoint_score_attribute="acc",
                                                    checkpoint_score_order="max")))
    r = trainer.fit()
    assert r.error is None
    kept = sorted(m["acc"] for _, m in r.best_checkpoints)
    # the two best (0.9, 0.8) plus the latest (0.2) survive; the rest are deleted from storage
    assert kept == [0.2, 0.8, 0.9]
    on_disk = [d for d in os.listdir(r.path) if d.startswith("checkpoint_")]
    assert len(on_disk) == 3
    with r.checkpoint.as_directory() as d:
        assert json.load(open(os.path.join(d, "state.json")))["epoch"] == 4
    assert list(r.metrics_dataframe["acc"]) == [0.1, 0.9, 0.4, 0.8, 0.2]


def _ctx_loop(config):
    ctx = train.get_context()
    train.report({"rank": ctx.get_world_rank(), "world": ctx.get_world_size(), "local": ctx.get_local_rank(),
                  "local_world": ctx.get_local_world_size(), "node_rank": ctx.get_node_rank(),
                  "experiment": ctx.get_experiment_name()})


def test_worker_context(ray_start_regular, tmp_path):
    r = TorchTrainer(_ctx_loop, scaling_config=ScalingConfig(num_workers=3),
                     run_config=RunConfig(name="ctxrun", storage_path=str(tmp_path))).fit()
    m = r.metrics
    assert m["rank"] == 0 and m["world"] == 3 and m["local_world"] == 3 and m["node_rank"] == 0
    assert m["experiment"] == "ctxrun"


def _loader_loop(config):
    from torch.utils.data import DataLoader, TensorDataset

    from ray_community_amd.train import torch as rt

    ds = TensorDataset(torch.arange(40).float())
    dl = rt.prepare_data_loader(DataLoader(ds, batch_size=5, shuffle=False))
    seen = sorted(int(x) for (b,) in dl for x in b)
    train.report({"seen": seen, "rank": train.get_context().get_world_rank()})
    # every rank reports; gather the shards through a collective to check the partition
    import torch.distributed as dist

    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, seen)
    train.report({"all": out})


def test_prepare_data_loader_shards_disjointly(ray_start_regular, tmp_path):
    r = TorchTrainer(_loader_loop, scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(name="dl", storage_path=str(tmp_path))).fit()
    a, b = r.metrics["all"]
    assert len(a) == len(b) == 20 and not set(a) & set(b) and sorted(a + b) == list(range(40))


def _resume_loop(config):
    start = 0
    ck = train.get_checkpoint()
    if ck:
        with ck.as_directory() as d:
            start = json.load(open(os.path.join(d, "s.json")))["epoch"] + 1
    for e in range(start, config["epochs"]):
        with tempfile.TemporaryDirectory() as d:
            json.dump({"epoch": e}, open(os.path.join(d, "s.json"), "w"))
            train.report({"epoch": e, "start": start}, checkpoint=Checkpoint.from_directory(d))


def test_restore_continues_from_latest_checkpoint(ray_start_regular, tmp_path):
    rc = RunConfig(name="resume", storage_path=str(tmp_path))
    r1 = TorchTrainer(_resume_loop, train_loop_config={"epochs": 2}, scaling_config=ScalingConfig(num_workers=1),
                      run_config=rc).fit()
    assert r1.metrics["epoch"] == 1
    assert TorchTrainer.can_restore(r1.path)
    t2 = TorchTrainer.restore(r1.path, train_loop_per_worker=_resume_loop, train_loop_config={"epochs": 4},
                              scaling_config=ScalingConfig(num_workers=1),
                              run_config=RunConfig(name="resume2", storage_path=str(tmp_path)))
    r2 = t2.fit()
    assert r2.metrics["epoch"] == 3 and r2.metrics["start"] == 2
