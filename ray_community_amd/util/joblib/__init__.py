"""joblib backend on the framework's process pool (reference: ``python/ray/util/joblib/``).

    from ray_community_amd.util.joblib import register_ray
    register_ray()
    with joblib.parallel_backend("ray"):
        Parallel(n_jobs=8)(delayed(f)(i) for i in range(100))
"""
from __future__ import annotations


def register_ray():
    try:
        from joblib.parallel import register_parallel_backend
    except ImportError as e:  # pragma: no cover
        raise ImportError("joblib is required for the 'ray' joblib backend") from e
    from .ray_backend import RayBackend

    register_parallel_backend("ray", RayBackend)
