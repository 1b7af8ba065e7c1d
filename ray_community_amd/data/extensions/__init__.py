"""``ray.data.extensions``: tensor column types for Arrow and pandas (see ``tensor_extension``)."""
from .tensor_extension import (ArrowTensorArray, ArrowTensorType, TensorArray, TensorDtype,  # noqa: F401
                               is_tensor_type, tensor_column_to_numpy)

__all__ = ["ArrowTensorArray", "ArrowTensorType", "TensorArray", "TensorDtype"]
