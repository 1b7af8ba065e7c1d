from .policy import PolicySpec
from .sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch, concat_samples

__all__ = ["SampleBatch", "MultiAgentBatch", "concat_samples", "DEFAULT_POLICY_ID", "PolicySpec"]
