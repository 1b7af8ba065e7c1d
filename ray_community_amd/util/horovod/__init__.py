"""``ray.util.horovod`` (reference: python/ray/util/horovod/): needs `horovod`, which is not installed in
this environment -- importing it fails the same way the reference's does without `horovod`."""
raise ImportError("ray_community_amd.util.horovod needs `horovod`, which is not installed in this environment")
