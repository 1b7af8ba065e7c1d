"""``ray.train.horovod`` (reference: python/ray/train/horovod/): needs `horovod`, which is not installed in
this environment. Torch training goes through ``ray_community_amd.train.torch``."""
raise ImportError("ray_community_amd.train.horovod needs `horovod`, which is not installed in this environment")
