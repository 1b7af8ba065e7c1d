"""SampleBatch (reference: ``rllib/policy/sample_batch.py``).

A dict of equally-long column arrays. Rollout fragments are kept time-major per env as
``[num_envs, T]`` blocks (``SampleBatch.fragment_shape``) so GAE runs as one batched HIP scan;
``concat_samples`` stacks fragments along the env axis and can run on device in one launch.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Optional

import numpy as np


class SampleBatch(dict):
    OBS = "obs"
    NEXT_OBS = "new_obs"
    ACTIONS = "actions"
    REWARDS = "rewards"
    TERMINATEDS = "terminateds"
    TRUNCATEDS = "truncateds"
    DONES = "dones"
    INFOS = "infos"
    EPS_ID = "eps_id"
    ENV_ID = "env_id"
    T = "t"
    ACTION_DIST_INPUTS = "action_dist_inputs"
    ACTION_LOGP = "action_logp"
    VF_PREDS = "vf_preds"
    VALUES_BOOTSTRAPPED = "values_bootstrapped"
    NEXT_VF_PREDS = "next_vf_preds"
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"
    SEQ_LENS = "seq_lens"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.fragment_shape = None  # (num_envs, T) when columns are env-major rollout blocks

    @property
    def count(self) -> int:
        for v in self.values():
            if hasattr(v, "shape") and len(v.shape) >= 1:
                if self.fragment_shape is not None:
                    return int(self.fragment_shape[0] * self.fragment_shape[1])
                return int(v.shape[0])
            if isinstance(v, list):
                return len(v)
        return 0

    def __len__(self):
        return self.count

    def env_steps(self):
        return self.count

    def agent_steps(self):
        return self.count

    def flatten(self) -> "SampleBatch":
        """[N, T, ...] fragment blocks -> [N*T, ...] rows."""
        if self.fragment_shape is None:
            return self
        N, T = self.fragment_shape
        out = SampleBatch()
        for k, v in self.items():
            if hasattr(v, "shape") and tuple(v.shape[:2]) == (N, T):
                out[k] = v.reshape((N * T,) + tuple(v.shape[2:]))
            else:
                out[k] = v
        return out

    def slice(self, start: int, end: int) -> "SampleBatch":
        return SampleBatch({k: v[start:end] for k, v in self.items()})

    def __getitem__(self, key):
        if isinstance(key, slice):
            return self.slice(key.start or 0, key.stop if key.stop is not None else self.count)
        v = dict.__getitem__(self, key)
        f = self._get_interceptor
        return f(v) if f is not None else v

    def shuffle(self, rng=None) -> "SampleBatch":
        n = self.count
        perm = (rng or np.random).permutation(n)
        for k, v in list(self.items()):
            if hasattr(v, "shape") and v.shape[:1] == (n,):
                self[k] = v[perm] if isinstance(v, np.ndarray) else v[_to_index(perm, v)]
        return self

    def timeslices(self, size: int) -> List["SampleBatch"]:
        return [self.slice(i, min(i + size, self.count)) for i in range(0, self.count, size)]

    def minibatches(self, size: int, rng=None) -> Iterator["SampleBatch"]:
        n = self.count
        perm = (rng or np.random).permutation(n)
        for i in range(0, n - size + 1 if n >= size else 1, size):
            idx = perm[i: i + size]
            yield SampleBatch({k: (v[idx] if isinstance(v, np.ndarray) else v[_to_index(idx, v)])
                               for k, v in self.items() if hasattr(v, "shape")})

    def copy(self, shallow=False):
        out = SampleBatch({k: (v if shallow else v.copy() if hasattr(v, "copy") else v) for k, v in self.items()})
        out.fragment_shape = self.fragment_shape
        return out

    def to_device(self, device):
        import warnings

        import torch

        out = SampleBatch()
        for k, v in self.items():
            if isinstance(v, np.ndarray) and v.dtype != object:
                with warnings.catch_warnings():
                    # fragments mapped from the shared-memory store are read-only by contract; the
                    # tensor made over them is only the source of this copy, never written
                    warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
                    t = torch.from_numpy(np.ascontiguousarray(v))
                out[k] = t.to(device, non_blocking=True)
            elif hasattr(v, "to"):
                out[k] = v.to(device)
            else:
                out[k] = v
        out.fragment_shape = self.fragment_shape
        return out

    def as_multi_agent(self, policy_id="default_policy"):
        return MultiAgentBatch({policy_id: self}, self.count)

    # ------------------------------------------------------------------ reference API surface
    # (rllib/policy/sample_batch.py: columns / rows / concat / split_by_episode / right_zero_pad /
    # compress / training flag / single-step input dicts)
    is_training = False
    zero_padded = False
    max_seq_len = None
    _slice_by_batch_id = False
    _get_interceptor = None

    def set_training(self, training: bool = True):
        self.is_training = bool(training)
        return self

    def columns(self, keys) -> List:
        return [self[k] for k in keys]

    def rows(self) -> Iterator[Dict]:
        """One dict per timestep (flattened fragment blocks; seq_lens and state columns skipped)."""
        flat = self.flatten()
        n = flat.count
        keys = [k for k in flat if k != SampleBatch.SEQ_LENS and not str(k).startswith("state_in")]
        for i in range(n):
            yield {k: flat[k][i] for k in keys}

    def size_bytes(self) -> int:
        tot = 0
        for v in self.values():
            if hasattr(v, "nbytes"):
                tot += int(v.nbytes)
            elif hasattr(v, "element_size"):
                tot += int(v.element_size() * v.numel())
        return tot

    def concat(self, other: "SampleBatch") -> "SampleBatch":
        return concat_samples([self, other])

    concat_samples = staticmethod(lambda batches: concat_samples(batches))

    def is_terminated_or_truncated(self) -> bool:
        flat = self.flatten()
        if flat.count == 0:
            return False
        for k in (SampleBatch.TERMINATEDS, SampleBatch.TRUNCATEDS, SampleBatch.DONES):
            if k in flat and bool(np.asarray(flat[k])[-1]):
                return True
        return False

    def is_single_trajectory(self) -> bool:
        """One episode (or a chunk of one): a single eps_id and no episode end before the last row."""
        flat = self.flatten()
        if SampleBatch.EPS_ID in flat and len(np.unique(np.asarray(flat[SampleBatch.EPS_ID]))) > 1:
            return False
        ends = np.zeros(flat.count, bool)
        for k in (SampleBatch.TERMINATEDS, SampleBatch.TRUNCATEDS, SampleBatch.DONES):
            if k in flat:
                ends |= np.asarray(flat[k], bool)
        return not ends[:-1].any()

    def split_by_episode(self, key: Optional[str] = None) -> List["SampleBatch"]:
        """Consecutive rows of one episode per batch: on changes of ``eps_id`` (or of ``key``), else
        after every terminated / truncated row."""
        flat = self.flatten()
        n = flat.count
        if n == 0:
            return []
        col = key or (SampleBatch.EPS_ID if SampleBatch.EPS_ID in flat else None)
        if col is not None and col in flat:
            ids = np.asarray(flat[col])
            cuts = list(np.nonzero(ids[1:] != ids[:-1])[0] + 1)
        else:
            ends = np.zeros(n, bool)
            for k in (SampleBatch.TERMINATEDS, SampleBatch.TRUNCATEDS, SampleBatch.DONES):
                if k in flat:
                    ends |= np.asarray(flat[k], bool)
            cuts = list(np.nonzero(ends[:-1])[0] + 1)
        bounds = [0] + cuts + [n]
        return [flat.slice(a, b) for a, b in zip(bounds[:-1], bounds[1:])]

    def right_zero_pad(self, max_seq_len: int, exclude_states: bool = True) -> "SampleBatch":
        """In place: every sequence (``seq_lens``) padded with zeros at its end to ``max_seq_len``
        rows; ``state_in_*`` columns (one row per sequence) stay as they are unless
        ``exclude_states=False``."""
        seq_lens = self.get(SampleBatch.SEQ_LENS)
        if seq_lens is None:
            raise ValueError("Cannot right-zero-pad a SampleBatch without a `seq_lens` column")
        lens = np.asarray(seq_lens, dtype=np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        for k in list(self.keys()):
            if k == SampleBatch.SEQ_LENS or (exclude_states and str(k).startswith("state_in")):
                continue
            v = self[k]
            if isinstance(v, list):
                v = np.asarray(v)
            if not hasattr(v, "shape") or v.shape[:1] != (int(lens.sum()),):
                continue
            out = np.zeros((len(lens) * max_seq_len,) + tuple(v.shape[1:]), dtype=v.dtype)
            for i, (s0, ln) in enumerate(zip(starts, lens)):
                out[i * max_seq_len: i * max_seq_len + ln] = v[s0: s0 + ln]
            self[k] = out
        self.zero_padded = True
        self.max_seq_len = int(max_seq_len)
        return self

    zero_pad = right_zero_pad

    def compress(self, bulk: bool = False, columns=frozenset(["obs", "new_obs"])) -> "SampleBatch":
        """In place: the given columns become zlib-compressed bytes (one blob per column with
        ``bulk``, else one per row), restored by ``decompress_if_needed``."""
        import pickle
        import zlib

        for k in columns:
            if k in self and isinstance(self[k], np.ndarray):
                v = self[k]
                if bulk:
                    self[k] = {"__zlib__": zlib.compress(pickle.dumps(v, protocol=5), 1)}
                else:
                    self[k] = np.array([zlib.compress(pickle.dumps(r, protocol=5), 1) for r in v], dtype=object)
        return self

    def decompress_if_needed(self, columns=frozenset(["obs", "new_obs"])) -> "SampleBatch":
        import pickle
        import zlib

        for k in columns:
            if k not in self:
                continue
            v = self[k]
            if isinstance(v, dict) and "__zlib__" in v:
                self[k] = pickle.loads(zlib.decompress(v["__zlib__"]))
            elif isinstance(v, np.ndarray) and v.dtype == object and len(v) and isinstance(v[0], bytes):
                self[k] = np.stack([pickle.loads(zlib.decompress(r)) for r in v])
        return self

    def get_single_step_input_dict(self, view_requirements=None, index="last") -> "SampleBatch":
        """A batch of one row (the last, or ``index``) with ``obs`` taken from that row's
        ``new_obs``: the input of the next forward pass after this trajectory."""
        flat = self.flatten()
        i = flat.count - 1 if index == "last" else int(index)
        out = SampleBatch({k: flat[k][i: i + 1] for k in flat if hasattr(flat[k], "shape") and k != SampleBatch.SEQ_LENS})
        if SampleBatch.NEXT_OBS in flat and index == "last":
            out[SampleBatch.OBS] = flat[SampleBatch.NEXT_OBS][i: i + 1]
        return out

    def enable_slicing_by_batch_id(self):
        self._slice_by_batch_id = True

    def disable_slicing_by_batch_id(self):
        self._slice_by_batch_id = False

    def set_get_interceptor(self, fn):
        """``fn(value)`` is applied to every column read through ``[key]`` (e.g. to move it to a
        device lazily)."""
        self._get_interceptor = fn


def _to_index(idx, v):
    import torch

    return torch.as_tensor(idx, device=v.device)


def concat_samples(batches: List[SampleBatch]) -> SampleBatch:
    """Concatenate batches. Fragment blocks with equal T stack along the env axis."""
    batches = [b for b in batches if b is not None and b.count > 0]
    if not batches:
        return SampleBatch()
    if isinstance(batches[0], MultiAgentBatch):
        return MultiAgentBatch.concat_samples(batches)
    fs = [b.fragment_shape for b in batches]
    out = SampleBatch()
    keys = batches[0].keys()
    if all(f is not None for f in fs) and len({f[1] for f in fs}) == 1:
        for k in keys:
            out[k] = _cat([b[k] for b in batches])
        out.fragment_shape = (sum(f[0] for f in fs), fs[0][1])
        return out
    flat = [b.flatten() for b in batches]
    for k in keys:
        out[k] = _cat([b[k] for b in flat])
    return out


def _cat(xs):
    if isinstance(xs[0], np.ndarray):
        return np.concatenate(xs, axis=0)
    import torch

    if isinstance(xs[0], torch.Tensor):
        from ...ops import batched_concat

        return batched_concat(xs)
    if isinstance(xs[0], list):
        return sum(xs, [])
    return xs[0]


class MultiAgentBatch:
    """Per-policy SampleBatches of one sampling round (reference ``MultiAgentBatch``)."""

    def __init__(self, policy_batches: Dict[str, SampleBatch], env_steps: int):
        self.policy_batches = policy_batches
        self._env_steps = env_steps
        self.fragment_shape = None

    def __getitem__(self, pid):
        return self.policy_batches[pid]

    def __contains__(self, pid):
        return pid in self.policy_batches

    def __len__(self):
        return self._env_steps

    @property
    def count(self):
        return self._env_steps

    def env_steps(self):
        return self._env_steps

    def agent_steps(self):
        return sum(b.count for b in self.policy_batches.values())

    @staticmethod
    def concat_samples(batches):
        pids = set()
        for b in batches:
            pids |= set(b.policy_batches)
        return MultiAgentBatch({p: concat_samples([b.policy_batches[p] for b in batches if p in b.policy_batches])
                                for p in pids}, sum(b.count for b in batches))


DEFAULT_POLICY_ID = "default_policy"
