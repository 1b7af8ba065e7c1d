"""``ray.air.data_batch_type``: what a batch of Data can be."""
from typing import Any, Dict, Union

import numpy as np

DataBatchType = Union[np.ndarray, Dict[str, np.ndarray], Any]  # + pandas.DataFrame / pyarrow.Table
