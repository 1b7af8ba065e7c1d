"""Hugging Face integrations (reference: ``python/ray/train/huggingface``): run a
``transformers.Trainer`` inside ``TorchTrainer`` workers -- ``transformers.prepare_trainer`` and
``transformers.RayTrainReportCallback``."""
