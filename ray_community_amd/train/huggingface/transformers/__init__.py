"""``transformers.Trainer`` inside a Train worker (reference:
``python/ray/train/huggingface/transformers/_transformers_utils.py``).

Run a normal ``transformers.Trainer`` in the ``train_loop_per_worker`` of a ``TorchTrainer``: the
worker group has already initialised ``torch.distributed`` (RCCL on GPUs, gloo on CPU) and set
``RANK/LOCAL_RANK/WORLD_SIZE``, so the Trainer runs data-parallel across the workers.
``RayTrainReportCallback`` forwards every save (metrics + checkpoint directory) to
``train.report``; ``prepare_trainer`` makes Trainer consume Data iterators from
``train.get_dataset_shard``.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from typing import Iterator

from transformers.trainer_callback import TrainerCallback

CHECKPOINT_DIR_NAME = "checkpoint"


class RayTrainReportCallback(TrainerCallback):
    CHECKPOINT_NAME = CHECKPOINT_DIR_NAME

    def __init__(self, *args, **kwargs):
        super().__init__()
        self._last_logs = {}

    def on_log(self, args, state, control, logs=None, **kwargs):
        if logs:
            self._last_logs.update({k: v for k, v in logs.items() if isinstance(v, (int, float))})

    def on_save(self, args, state, control, **kwargs):
        from ... import Checkpoint, report

        metrics = dict(self._last_logs)
        for log in state.log_history:
            metrics.update({k: v for k, v in log.items() if isinstance(v, (int, float))})
        metrics["step"] = state.global_step
        metrics["epoch"] = state.epoch
        src = os.path.join(args.output_dir, f"checkpoint-{state.global_step}")
        with tempfile.TemporaryDirectory() as tmp:
            ckpt = None
            if os.path.isdir(src):
                dst = os.path.join(tmp, self.CHECKPOINT_NAME)
                shutil.copytree(src, dst)
                ckpt = Checkpoint.from_directory(dst)
            report(metrics, checkpoint=ckpt)


class RayTorchIterableDataset:
    """Wraps a Data iterator (``iter_torch_batches`` / ``iter_rows``) as a torch IterableDataset."""

    def __init__(self, data_iterable) -> None:
        from torch.utils.data import IterableDataset

        self._it = data_iterable
        self.__class__ = type("RayTorchIterableDataset", (RayTorchIterableDataset, IterableDataset), {})

    def __iter__(self) -> Iterator:
        return iter(self._it)


def prepare_trainer(trainer):
    """Let ``trainer`` take framework Data iterators (from ``get_dataset_shard``) as datasets."""
    from torch.utils.data import DataLoader

    base = trainer.__class__

    class _RayTrainer(base):
        def get_train_dataloader(self):
            ds = self.train_dataset
            if hasattr(ds, "iter_torch_batches"):
                it = ds.iter_torch_batches(batch_size=self.args.per_device_train_batch_size)
                return DataLoader(RayTorchIterableDataset(it), batch_size=None)
            return super().get_train_dataloader()

        def get_eval_dataloader(self, eval_dataset=None):
            ds = eval_dataset if eval_dataset is not None else self.eval_dataset
            if hasattr(ds, "iter_torch_batches"):
                it = ds.iter_torch_batches(batch_size=self.args.per_device_eval_batch_size)
                return DataLoader(RayTorchIterableDataset(it), batch_size=None)
            return super().get_eval_dataloader(eval_dataset)

    trainer.__class__ = _RayTrainer
    return trainer


__all__ = ["RayTrainReportCallback", "prepare_trainer", "RayTorchIterableDataset"]
