"""``ray.train.lightgbm`` (reference: ``python/ray/train/lightgbm/``): ``LightGBMTrainer``,
``RayTrainReportCallback``, ``LightGBMCheckpoint``, ``LightGBMPredictor``.

lightgbm is not on this platform; the trainer runs the native data-parallel histogram GBDT
(``train/gbdt``) with lightgbm's parameter names and defaults: leaf-wise (``lossguide``) growth
with ``num_leaves`` 31, ``learning_rate`` 0.1, ``min_data_in_leaf`` 20,
``min_sum_hessian_in_leaf`` 1e-3, ``lambda_l2`` 0, ``max_bin`` 255, ``feature_fraction`` /
``bagging_fraction``; objectives ``regression``, ``binary``, ``multiclass``; metrics ``l2``,
``l1``, ``rmse``, ``binary_logloss``, ``binary_error``, ``multi_logloss``, ``multi_error``.
"""
from ..gbdt.core import Booster, DMatrix
from ..gbdt.core import train as _train
from ..gbdt.trainer import GBDTCheckpoint, GBDTConfig, GBDTPredictor, _GBDTTrainer
from ..gbdt.trainer import RayTrainReportCallback as _Report


def train(params, train_set, num_boost_round=100, valid_sets=(), valid_names=None, init_model=None,
          callbacks=(), **kw):
    """``lightgbm.train``-shaped entry point on the native engine."""
    names = list(valid_names or [f"valid_{i}" for i in range(len(valid_sets))])
    return _train(params, train_set, num_boost_round, evals=list(zip(valid_sets, names)), xgb_model=init_model,
                  callbacks=callbacks, flavor="lightgbm", **kw)


Dataset = DMatrix


class RayTrainReportCallback(_Report):
    pass


class LightGBMCheckpoint(GBDTCheckpoint):
    pass


class LightGBMConfig(GBDTConfig):
    """Worker-group backend for ``LightGBMTrainer(train_loop_per_worker, ...)``."""


class LightGBMPredictor(GBDTPredictor):
    pass


class LightGBMTrainer(_GBDTTrainer):
    """Data-parallel leaf-wise boosting over the ``"train"`` dataset's shards (see module doc)."""

    _flavor = "lightgbm"

    @classmethod
    def _report_callback_cls(cls):
        return RayTrainReportCallback


__all__ = ["LightGBMTrainer", "RayTrainReportCallback", "LightGBMCheckpoint", "LightGBMConfig", "LightGBMPredictor", "Booster",
           "Dataset", "train"]
