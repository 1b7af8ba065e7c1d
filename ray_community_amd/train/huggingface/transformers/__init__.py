"""``transformers.Trainer`` inside Ray Train workers (reference:
``python/ray/train/huggingface/transformers/_transformers_utils.py``).

* ``RayTrainReportCallback``: after every checkpoint the HF Trainer saves, report the merged log
  history as metrics together with a copy of that checkpoint (under ``checkpoint/`` in the Ray
  Train checkpoint directory), so ``RunConfig`` / ``CheckpointConfig`` keep and rank them;
* ``prepare_trainer``: let the Trainer consume Ray Data shards directly -- a dataset given as
  ``get_dataset_shard(...).iter_torch_batches(...)`` (already batched, re-iterable per epoch) is
  served by a pass-through DataLoader instead of HF's sampler / collator.

The process group is the one ``TorchTrainer`` set up (RCCL on GPUs, gloo on CPU): the HF Trainer
finds ``torch.distributed`` initialised and uses it.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from typing import Optional

try:
    import transformers
    from transformers.trainer_callback import TrainerCallback
    _IMPORT_ERROR: Optional[ImportError] = None
except ImportError as e:  # pragma: no cover - transformers is optional
    transformers = None
    TrainerCallback = object
    _IMPORT_ERROR = e


class RayTrainReportCallback(TrainerCallback):
    CHECKPOINT_NAME = "checkpoint"

    def on_save(self, args, state, control, **kwargs):
        from ... import Checkpoint, report
        from transformers.trainer_utils import get_last_checkpoint

        metrics = {}
        for entry in state.log_history:  # later entries win (the latest loss / eval metrics)
            metrics.update(entry)
        metrics.setdefault("step", state.global_step)
        metrics.setdefault("epoch", state.epoch)
        src = get_last_checkpoint(args.output_dir) if os.path.isdir(args.output_dir) else None
        if src is None:
            report(metrics)
            return
        with tempfile.TemporaryDirectory() as tmp:
            shutil.copytree(src, os.path.join(tmp, self.CHECKPOINT_NAME))
            report(metrics, checkpoint=Checkpoint.from_directory(tmp))


def _is_ray_iterable(ds) -> bool:
    from ....data.iterator import _IterableFromIterator

    return isinstance(ds, _IterableFromIterator)


def prepare_trainer(trainer):
    """Return ``trainer`` (same object) with data loaders that accept Ray Data iterables."""
    if _IMPORT_ERROR is not None:
        raise _IMPORT_ERROR
    from torch.utils.data import DataLoader, IterableDataset

    class _Batches(IterableDataset):
        def __init__(self, it):
            super().__init__()
            self.it = it

        def __iter__(self):
            return iter(self.it)

    def _loader(ds):
        # batches arrive formed: a batch_size=1 loader that unwraps them
        return DataLoader(_Batches(ds), batch_size=1, collate_fn=lambda items: items[0])

    base = type(trainer)

    class RayTransformersTrainer(base):
        def get_train_dataloader(self):
            if _is_ray_iterable(self.train_dataset):
                return _loader(self.train_dataset)
            return super().get_train_dataloader()

        def get_eval_dataloader(self, eval_dataset=None):
            ds = self.eval_dataset if eval_dataset is None else eval_dataset
            if _is_ray_iterable(ds):
                return _loader(ds)
            return super().get_eval_dataloader(eval_dataset)

    RayTransformersTrainer.__name__ = f"Ray{base.__name__}"
    trainer.__class__ = RayTransformersTrainer
    return trainer


__all__ = ["RayTrainReportCallback", "prepare_trainer"]
