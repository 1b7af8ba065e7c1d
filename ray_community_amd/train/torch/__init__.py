from .config import TorchConfig
from .torch_checkpoint import TorchCheckpoint, TorchDetectionPredictor, TorchPredictor
from .torch_trainer import TorchTrainer
from .train_loop_utils import (accelerate, backward, enable_reproducibility, get_device, get_devices, prepare_data_loader,
                               prepare_model, prepare_optimizer, TorchWorkerProfiler)

__all__ = ["TorchTrainer", "TorchConfig", "prepare_model", "prepare_data_loader", "prepare_optimizer", "get_device",
           "get_devices", "accelerate", "backward", "enable_reproducibility", "TorchCheckpoint", "TorchPredictor",
           "TorchDetectionPredictor", "TorchWorkerProfiler"]
