"""transformers.Trainer under TorchTrainer (reference tests:
python/ray/train/tests/test_transformers_trainer.py). Tiny randomly initialised GPT-2 (no
downloads possible), 2 CPU workers over gloo."""
import pytest

import ray_community_amd as ray
from ray_community_amd.train import RunConfig, ScalingConfig
from ray_community_amd.train.torch import TorchTrainer


def _loop(config):
    import torch
    from transformers import GPT2Config, GPT2LMHeadModel, Trainer, TrainingArguments

    from ray_community_amd import train
    from ray_community_amd.train.huggingface.transformers import RayTrainReportCallback, prepare_trainer

    torch.manual_seed(0)
    model = GPT2LMHeadModel(GPT2Config(n_layer=2, n_head=2, n_embd=32, vocab_size=64, n_positions=32))

    class DS(torch.utils.data.Dataset):
        def __len__(self):
            return 64

        def __getitem__(self, i):
            x = torch.arange(16) % 8 + (i % 4)
            return {"input_ids": x, "labels": x}

    args = TrainingArguments(output_dir=config["out"], per_device_train_batch_size=4, max_steps=8,
                             save_steps=4, logging_steps=2, report_to=[], use_cpu=True, learning_rate=1e-3,
                             save_strategy="steps", disable_tqdm=True)
    trainer = Trainer(model=model, args=args, train_dataset=DS(), callbacks=[RayTrainReportCallback()])
    trainer = prepare_trainer(trainer)
    trainer.train()
    train.report({"world": train.get_context().get_world_size()})


def test_transformers_trainer_on_two_workers(shutdown_only, tmp_path):
    ray.init(num_cpus=4)
    trainer = TorchTrainer(_loop, train_loop_config={"out": str(tmp_path / "hf_out")},
                           scaling_config=ScalingConfig(num_workers=2),
                           run_config=RunConfig(name="hf", storage_path=str(tmp_path)))
    result = trainer.fit()
    assert result.error is None
    assert result.checkpoint is not None
    assert result.metrics["world"] == 2
