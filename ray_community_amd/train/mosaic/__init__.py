"""``ray.train.mosaic`` (reference: python/ray/train/mosaic/): needs `composer`, which is not installed in
this environment. Torch training goes through ``ray_community_amd.train.torch``."""
raise ImportError("ray_community_amd.train.mosaic needs `composer`, which is not installed in this environment")
