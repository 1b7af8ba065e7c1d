"""Off-policy estimator base (reference: ``rllib/offline/estimators/off_policy_estimator.py``)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

from ...policy.sample_batch import SampleBatch


def split_by_episode(batch: SampleBatch, complete_only: bool = False) -> List[SampleBatch]:
    """Episodes of a batch: by ``eps_id`` when present (an env-major ``[N, T]`` fragment is
    flattened row by row first, so each episode's steps stay in order), else env-major fragments
    are cut per env row at terminated / truncated steps and flat batches at the done flags.
    ``complete_only``: drop pieces that do not end in a terminated / truncated step (cut off by
    the end of the logged data)."""
    fs = getattr(batch, "fragment_shape", None)
    if SampleBatch.EPS_ID in batch:
        if fs is not None:
            N, T = fs
            batch = SampleBatch({k: np.asarray(v).reshape((N * T,) + np.asarray(v).shape[2:]) for k, v in batch.items()
                                 if isinstance(v, np.ndarray) and v.ndim >= 2 and v.shape[:2] == (N, T)})
        ids = np.asarray(batch[SampleBatch.EPS_ID])
        out = []
        for e in dict.fromkeys(ids.tolist()):
            m = ids == e
            out.append(SampleBatch({k: np.asarray(v)[m] for k, v in batch.items() if isinstance(v, np.ndarray)}))
        return [e for e in out if not complete_only or _ends_done(e)]
    rows = []
    if fs is not None:
        N, T = fs
        for i in range(N):
            rows.append(SampleBatch({k: np.asarray(v)[i] for k, v in batch.items()
                                     if isinstance(v, np.ndarray) and v.ndim >= 2 and v.shape[:2] == (N, T)}))
    else:
        rows = [batch]
    out = []
    for r in rows:
        n = len(r[SampleBatch.REWARDS])
        done = np.asarray(r.get(SampleBatch.TERMINATEDS, np.zeros(n, bool)), bool)
        if SampleBatch.TRUNCATEDS in r:
            done = done | np.asarray(r[SampleBatch.TRUNCATEDS], bool)
        s = 0
        for t in np.nonzero(done)[0].tolist() + ([n - 1] if n and not done[-1] else []):
            out.append(SampleBatch({k: np.asarray(v)[s: t + 1] for k, v in r.items()}))
            s = t + 1
    return [e for e in out if len(e[SampleBatch.REWARDS]) and (not complete_only or _ends_done(e))]


def _ends_done(ep: SampleBatch) -> bool:
    last = bool(np.asarray(ep.get(SampleBatch.TERMINATEDS, [False]))[-1])
    if SampleBatch.TRUNCATEDS in ep:
        last = last or bool(np.asarray(ep[SampleBatch.TRUNCATEDS])[-1])
    return last


class OffPolicyEstimator:
    """``policy``: anything with a torch ``module`` (RLModule) or ``model`` attribute, an
    ``Algorithm`` (its current module), or an RLModule itself. ``gamma``: discount of both
    estimates. ``epsilon_greedy``: the target policy is evaluated as epsilon-greedy over its
    greedy action instead of its own distribution (reference semantics)."""

    def __init__(self, policy, gamma: float = 0.99, epsilon_greedy: float = 0.0):
        self.module = _module_of(policy)
        self.gamma = float(gamma)
        self.epsilon_greedy = float(epsilon_greedy)

    # ------------------------------------------------------------------ probabilities
    @torch.no_grad()
    def action_probs_all(self, obs) -> np.ndarray:
        """pi(. | s) for a discrete action space: [B, A]."""
        o = torch.as_tensor(np.asarray(obs))
        logits, _ = self.module.forward(o)
        p = torch.softmax(logits.float(), -1).numpy()
        if self.epsilon_greedy > 0:
            A = p.shape[-1]
            g = np.zeros_like(p)
            g[np.arange(len(p)), p.argmax(-1)] = 1.0
            p = (1 - self.epsilon_greedy) * g + self.epsilon_greedy / A
        return p

    def compute_action_probs(self, batch: SampleBatch) -> np.ndarray:
        p = self.action_probs_all(batch[SampleBatch.OBS])
        a = np.asarray(batch[SampleBatch.ACTIONS]).astype(np.int64)
        return p[np.arange(len(a)), a]

    @staticmethod
    def behavior_probs(batch: SampleBatch) -> np.ndarray:
        if "action_prob" in batch:
            return np.asarray(batch["action_prob"], np.float64)
        if SampleBatch.ACTION_LOGP in batch:
            return np.exp(np.asarray(batch[SampleBatch.ACTION_LOGP], np.float64))
        raise ValueError("off-policy estimation needs the behavior policy's action_prob or action_logp")

    # ------------------------------------------------------------------ estimates
    def estimate_on_single_episode(self, episode: SampleBatch) -> Dict[str, float]:
        raise NotImplementedError

    def estimate(self, batch: SampleBatch, split_batch_by_episode: bool = True) -> Dict[str, float]:
        eps = split_by_episode(batch) if split_batch_by_episode else [batch]
        return self.estimate_episodes(eps)

    def estimate_episodes(self, eps: List[SampleBatch]) -> Dict[str, float]:
        rows = self.estimate_on_episodes(eps)
        vb = np.array([r["v_behavior"] for r in rows])
        vt = np.array([r["v_target"] for r in rows])
        return {"v_behavior": float(vb.mean()), "v_behavior_std": float(vb.std()), "v_target": float(vt.mean()),
                "v_target_std": float(vt.std()), "v_gain": float(vt.mean() / vb.mean()) if vb.mean() else float("nan"),
                "v_delta": float(vt.mean() - vb.mean()), "num_episodes": len(rows)}

    def estimate_on_episodes(self, episodes: List[SampleBatch]) -> List[Dict[str, float]]:
        return [self.estimate_on_single_episode(e) for e in episodes]

    def train(self, batch: SampleBatch) -> Dict:
        """Model-based estimators fit their model here (no-op for IS / WIS)."""
        return {}

    def _discounts(self, n):
        return self.gamma ** np.arange(n)


def _module_of(policy):
    if isinstance(policy, torch.nn.Module):
        return policy
    for attr in ("module", "model"):
        m = getattr(policy, attr, None)
        if isinstance(m, torch.nn.Module):
            return m
    get = getattr(policy, "get_module", None)
    if get is not None:
        return get()
    raise TypeError(f"cannot find a torch module in {type(policy).__name__}")
