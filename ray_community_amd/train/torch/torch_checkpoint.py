"""``TorchCheckpoint`` and ``TorchPredictor`` (reference: ``train/torch/torch_checkpoint.py``,
``torch_predictor.py``): a directory checkpoint holding a model's ``state_dict`` (``model.pt``) or
a whole module, and batch inference with it on numpy / pandas batches (``map_batches`` friendly)."""
from __future__ import annotations

import os
import tempfile
from typing import Any, Dict, Optional

import numpy as np

from .._checkpoint import Checkpoint

MODEL_KEY = "model.pt"


class TorchCheckpoint(Checkpoint):
    @classmethod
    def from_state_dict(cls, state_dict: Dict[str, Any], *, preprocessor=None) -> "TorchCheckpoint":
        import torch

        d = tempfile.mkdtemp(prefix="rca_torch_ckpt_")
        torch.save({k: v.detach().cpu() if hasattr(v, "detach") else v for k, v in state_dict.items()},
                   os.path.join(d, MODEL_KEY))
        ck = cls(d)
        if preprocessor is not None:
            ck._save_preprocessor(preprocessor)
        return ck

    @classmethod
    def from_model(cls, model, *, preprocessor=None) -> "TorchCheckpoint":
        import torch

        d = tempfile.mkdtemp(prefix="rca_torch_ckpt_")
        m = getattr(model, "module", model)  # unwrap DDP
        torch.save(m, os.path.join(d, MODEL_KEY))
        ck = cls(d)
        if preprocessor is not None:
            ck._save_preprocessor(preprocessor)
        return ck

    def _save_preprocessor(self, pre):
        import cloudpickle

        with open(os.path.join(self.path, "preprocessor.pkl"), "wb") as f:
            cloudpickle.dump(pre, f)

    def get_preprocessor(self):
        p = os.path.join(self.path, "preprocessor.pkl")
        if not os.path.exists(p):
            return None
        import cloudpickle

        with open(p, "rb") as f:  # written by this class (from_model / from_state_dict)
            return cloudpickle.load(f)

    def get_model(self, model=None):
        """The saved module, or ``model`` with the saved state dict loaded into it."""
        import torch

        obj = torch.load(os.path.join(self.path, MODEL_KEY), map_location="cpu", weights_only=False)
        if isinstance(obj, torch.nn.Module):
            return obj
        if model is None:
            raise ValueError("this checkpoint holds a state_dict: pass the model to load it into")
        model.load_state_dict(obj)
        return model


class TorchPredictor:
    """Batch inference with a torch module (on ``device``, default the GPU when present)."""

    def __init__(self, model, preprocessor=None, use_gpu: bool = False):
        import torch

        self.device = torch.device("cuda" if use_gpu and torch.cuda.is_available() else "cpu")
        self.model = model.to(self.device).eval()
        self.preprocessor = preprocessor

    @classmethod
    def from_checkpoint(cls, checkpoint: TorchCheckpoint, model=None, use_gpu: bool = False) -> "TorchPredictor":
        ck = checkpoint if isinstance(checkpoint, TorchCheckpoint) else TorchCheckpoint(checkpoint.path)
        return cls(ck.get_model(model), ck.get_preprocessor(), use_gpu)

    def _run(self, x):
        import torch

        with torch.no_grad():
            return self.model(x)

    def predict(self, data, dtype=None) -> Dict[str, np.ndarray]:
        """``data``: ndarray, dict of ndarrays (one model input each) or a pandas DataFrame
        (all columns stacked as features). Returns ``{"predictions": ndarray}``."""
        import torch

        if self.preprocessor is not None:
            data = self.preprocessor.transform_batch(data)
        if hasattr(data, "to_numpy") and not isinstance(data, np.ndarray):
            data = data.to_numpy()
        if isinstance(data, dict):
            ins = {k: torch.as_tensor(np.asarray(v), dtype=dtype, device=self.device) for k, v in data.items()}
            out = self._run(next(iter(ins.values())) if len(ins) == 1 else ins)
        else:
            out = self._run(torch.as_tensor(np.asarray(data), dtype=dtype, device=self.device))
        if isinstance(out, dict):
            return {k: v.cpu().numpy() for k, v in out.items()}
        return {"predictions": out.cpu().numpy()}


class TorchDetectionPredictor(TorchPredictor):
    """Detection models return a list of per-image dicts; predictions become dict columns."""

    def predict(self, data, dtype=None):
        import torch

        imgs = data["image"] if isinstance(data, dict) else data
        with torch.no_grad():
            outs = self.model([torch.as_tensor(np.asarray(i), dtype=dtype, device=self.device) for i in imgs])
        keys = outs[0].keys() if outs else []
        return {k: np.array([o[k].cpu().numpy() for o in outs], dtype=object) for k in keys}
