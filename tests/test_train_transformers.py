"""transformers.Trainer inside TorchTrainer workers (reference:
python/ray/train/huggingface/transformers, tests/test_transformers_trainer.py): Ray Data shards
feed the HF Trainer through prepare_trainer, and RayTrainReportCallback reports each HF checkpoint
with the merged log history. Tiny random-init GPT-2, CPU workers over gloo."""
import os

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import data as rd
from ray_community_amd import train
from ray_community_amd.train import RunConfig, ScalingConfig
from ray_community_amd.train.torch import TorchTrainer

transformers = pytest.importorskip("transformers")


def _loop(config):
    import torch
    from transformers import GPT2Config, GPT2LMHeadModel, Trainer, TrainingArguments

    from ray_community_amd.train.huggingface.transformers import RayTrainReportCallback, prepare_trainer

    torch.manual_seed(0)
    model = GPT2LMHeadModel(GPT2Config(vocab_size=64, n_positions=32, n_embd=32, n_layer=1, n_head=2,
                                                bos_token_id=0, eos_token_id=0))
    shard = train.get_dataset_shard("train")
    batches = shard.iter_torch_batches(batch_size=4, device="cpu",
                                       collate_fn=lambda b: {"input_ids": torch.as_tensor(b["ids"]),
                                                             "labels": torch.as_tensor(b["ids"])})
    args = TrainingArguments(output_dir=config["out"], max_steps=4, save_strategy="steps", save_steps=2,
                             logging_steps=1, per_device_train_batch_size=4, report_to=[], use_cpu=True,
                             disable_tqdm=True)
    trainer = Trainer(model=model, args=args, train_dataset=batches, callbacks=[RayTrainReportCallback()])
    trainer = prepare_trainer(trainer)
    assert type(trainer).__name__ == "RayTrainer"
    trainer.train()


def test_hf_trainer_reports_checkpoints_through_ray_train(shutdown_only, tmp_path):
    ray.init(num_cpus=4)
    ids = np.random.default_rng(0).integers(0, 64, (64, 16)).astype(np.int64)
    ds = rd.from_items([{"ids": r} for r in ids])
    trainer = TorchTrainer(_loop, train_loop_config={"out": str(tmp_path / "hf")},
                           scaling_config=ScalingConfig(num_workers=2, use_gpu=False),
                           datasets={"train": ds},
                           run_config=RunConfig(name="hf", storage_path=str(tmp_path / "ray")))
    result = trainer.fit()
    assert result.error is None
    m = result.metrics
    assert m["step"] == 4 and ("loss" in m or "train_loss" in m), m
    with result.checkpoint.as_directory() as d:
        inner = os.path.join(d, "checkpoint")
        files = set(os.listdir(inner))
        assert "model.safetensors" in files and "trainer_state.json" in files, files
