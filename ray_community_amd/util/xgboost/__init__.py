"""Removed API (reference: python/ray/util/xgboost/__init__.py raises on import)."""
raise DeprecationWarning("ray.util.xgboost has been removed as of Ray 2.0: use `XGBoostTrainer` in `ray.train.xgboost`.")
