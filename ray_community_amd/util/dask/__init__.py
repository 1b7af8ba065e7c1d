"""``ray.util.dask`` (reference: python/ray/util/dask/): needs `dask`, which is not installed in
this environment -- importing it fails the same way the reference's does without `dask`."""
raise ImportError("ray_community_amd.util.dask needs `dask`, which is not installed in this environment")
