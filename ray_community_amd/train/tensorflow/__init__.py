"""``ray.train.tensorflow`` (reference: python/ray/train/tensorflow/): needs `tensorflow`, which is not installed in
this environment. Torch training goes through ``ray_community_amd.train.torch``."""
raise ImportError("ray_community_amd.train.tensorflow needs `tensorflow`, which is not installed in this environment")
