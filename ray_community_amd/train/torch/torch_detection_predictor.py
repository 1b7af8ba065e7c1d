"""TorchDetectionPredictor (reference: train/torch/torch_detection_predictor.py): a
TorchPredictor for detection models whose forward returns one dict per image
(``boxes`` / ``labels`` / ``scores``, torchvision's convention). Images go in as a list / array of
CHW tensors; predictions come back as object arrays, one entry per image."""
from __future__ import annotations

from typing import Dict

import numpy as np

from .torch_checkpoint import TorchPredictor


class TorchDetectionPredictor(TorchPredictor):
    def predict(self, data, dtype=None) -> Dict[str, np.ndarray]:
        import torch

        if self.preprocessor is not None:
            data = self.preprocessor.transform_batch(data)
        images = data["image"] if isinstance(data, dict) else data
        batch = [torch.as_tensor(np.asarray(im), dtype=dtype or torch.float32, device=self.device) for im in images]
        with torch.no_grad():
            outs = self.model(batch)
        res: Dict[str, np.ndarray] = {}
        for key in ("boxes", "labels", "scores"):
            col = np.empty(len(outs), dtype=object)
            for i, o in enumerate(outs):
                col[i] = o[key].detach().cpu().numpy()
            res[f"pred_{key}"] = col
        return res
