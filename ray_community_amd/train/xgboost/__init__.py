"""``ray.train.xgboost`` (reference: ``python/ray/train/xgboost/``): ``XGBoostTrainer``,
``RayTrainReportCallback``, ``XGBoostCheckpoint``, ``XGBoostPredictor``.

The xgboost library is not on this platform; the trainer runs the same data-parallel histogram
algorithm natively (``train/gbdt``: quantile sketch, HIP histogram kernel, all-reduced histograms,
depthwise growth) and accepts xgboost's parameter names and defaults (``eta`` 0.3, ``max_depth`` 6,
``lambda`` 1, ``min_child_weight`` 1, ``max_bin`` 256; objectives ``reg:squarederror``,
``binary:logistic``, ``binary:logitraw``, ``multi:softprob``, ``multi:softmax``; metrics rmse,
mae, logloss, error, mlogloss, merror). Models are this framework's JSON format, not xgboost's.
"""
from ..gbdt.core import Booster, DMatrix, train
from ..gbdt.trainer import GBDTCheckpoint, GBDTConfig, GBDTPredictor, _GBDTTrainer
from ..gbdt.trainer import RayTrainReportCallback as _Report


class RayTrainReportCallback(_Report):
    pass


class XGBoostCheckpoint(GBDTCheckpoint):
    pass


class XGBoostConfig(GBDTConfig):
    """Worker-group backend for the v2 form ``XGBoostTrainer(train_loop_per_worker, ...)``."""


class XGBoostPredictor(GBDTPredictor):
    pass


class XGBoostTrainer(_GBDTTrainer):
    """Data-parallel boosting over the ``"train"`` dataset's shards; every other dataset is an eval
    set reported as ``{name}-{metric}``. ``num_boost_round`` is the TARGET number of trees (a
    resumed model trains only the remaining rounds). The reference's v2 form also works: pass a
    ``train_loop_per_worker`` (it calls ``ray.train.xgboost.train(..., callbacks=[
    RayTrainReportCallback()])`` on its ``get_dataset_shard`` data) plus ``xgboost_config``."""

    _flavor = "xgboost"

    @classmethod
    def _report_callback_cls(cls):
        return RayTrainReportCallback


__all__ = ["XGBoostTrainer", "RayTrainReportCallback", "XGBoostCheckpoint", "XGBoostConfig", "XGBoostPredictor", "Booster",
           "DMatrix", "train"]
