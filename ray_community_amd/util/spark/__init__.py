"""``ray.util.spark`` (reference: python/ray/util/spark/): needs `pyspark`, which is not installed in
this environment -- importing it fails the same way the reference's does without `pyspark`."""
raise ImportError("ray_community_amd.util.spark needs `pyspark`, which is not installed in this environment")
