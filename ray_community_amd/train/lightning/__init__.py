"""``ray.train.lightning`` (reference: python/ray/train/lightning/): needs `lightning`, which is not installed in
this environment. Torch training goes through ``ray_community_amd.train.torch``."""
raise ImportError("ray_community_amd.train.lightning needs `lightning`, which is not installed in this environment")
