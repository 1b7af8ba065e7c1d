from .policy import Policy, PolicySpec, TFPolicy, TorchPolicy, build_policy_class, build_tf_policy
from .sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch, concat_samples

__all__ = ["SampleBatch", "MultiAgentBatch", "concat_samples", "DEFAULT_POLICY_ID", "PolicySpec", "Policy",
           "TorchPolicy", "TFPolicy", "build_policy_class", "build_tf_policy"]
