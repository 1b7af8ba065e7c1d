"""Removed API (reference: python/ray/util/lightgbm/__init__.py raises on import)."""
raise DeprecationWarning("ray.util.lightgbm has been removed as of Ray 2.0: use `LightGBMTrainer` in `ray.train.lightgbm`.")
