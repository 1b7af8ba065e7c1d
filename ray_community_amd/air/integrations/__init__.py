"""Experiment-tracking integrations (reference: python/ray/air/integrations/{wandb,mlflow,comet}.py).

Weights & Biases, MLflow and Comet clients are not installed in this environment: the
callbacks and setup functions raise ImportError naming the missing package when used, so code
importing them still loads. TensorBoard logging works without extra packages
(``ray_community_amd.tune.logger.TBXLoggerCallback``)."""
