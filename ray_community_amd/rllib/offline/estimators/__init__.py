"""Off-policy estimation (reference: ``rllib/offline/estimators``): the value a TARGET policy would
get, estimated from episodes logged under a BEHAVIOR policy whose action probabilities were
recorded (``action_logp`` or ``action_prob``).

* ``ImportanceSampling`` (IS, ``importance_sampling.py:17``): per-decision cumulative ratios;
* ``WeightedImportanceSampling`` (WIS, ``weighted_importance_sampling.py:19``): the ratios
  normalised by their mean over the batch's episodes at each timestep;
* ``DirectMethod`` (DM, ``direct_method.py:23``): V(s_0) of a fitted-Q-evaluation model;
* ``DoublyRobust`` (DR, ``doubly_robust.py:28``): the FQE baseline corrected by IS residuals.
"""
from .direct_method import DirectMethod
from .doubly_robust import DoublyRobust
from .fqe_torch_model import FQETorchModel
from .importance_sampling import ImportanceSampling
from .off_policy_estimator import OffPolicyEstimator, split_by_episode
from .weighted_importance_sampling import WeightedImportanceSampling

__all__ = ["OffPolicyEstimator", "ImportanceSampling", "WeightedImportanceSampling", "DirectMethod",
           "DoublyRobust", "FQETorchModel", "split_by_episode"]
