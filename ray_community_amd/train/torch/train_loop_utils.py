"""Torch train-loop helpers (reference: ``python/ray/train/torch/train_loop_utils.py``)."""
from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional

import torch


def get_device() -> torch.device:
    idx = os.environ.get("RCA_TRAIN_DEVICE_INDEX")
    if torch.cuda.is_available():
        if idx is not None:
            return torch.device("cuda", int(idx))
        lr = os.environ.get("LOCAL_RANK")
        if lr is not None and int(lr) < torch.cuda.device_count():
            return torch.device("cuda", int(lr))
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def get_devices():
    return [get_device()]


def _world():
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


class _Accelerator:
    """Per-worker training optimizations (reference ``_TorchAccelerator``,
    ``train/torch/train_loop_utils.py:356``). ``amp``: the model's forward runs under
    ``torch.autocast``. On MI355X the autocast dtype defaults to bf16 -- the matrix cores' native
    16-bit input, with fp32's exponent range, so no loss scaling is needed and no GradScaler is
    built; ``dtype=torch.float16`` gives the reference's fp16 + GradScaler behaviour."""

    def __init__(self, amp: bool = False, dtype: Optional[torch.dtype] = None):
        self.amp_is_enabled = bool(amp)
        self.dtype = dtype or torch.bfloat16
        if self.dtype not in (torch.bfloat16, torch.float16):
            raise ValueError(f"autocast dtype must be torch.bfloat16 or torch.float16, got {self.dtype}")
        self.device_type = get_device().type
        self.scaler = None
        if self.amp_is_enabled and self.dtype == torch.float16:
            self.scaler = torch.amp.GradScaler(self.device_type)
        self._seed: Optional[int] = None


_ACCEL: Dict[str, Optional[_Accelerator]] = {"explicit": None, "default": None}


def _set_accelerator(acc: _Accelerator):
    from .._internal.session import _SESSION

    holder = _SESSION if _SESSION is not None else None
    if holder is not None:
        if getattr(holder, "_accelerator", None) is not None:
            raise RuntimeError("An accelerator has already been set. Make sure `train.torch.accelerate()` is not "
                               "called multiple times, and is called before any of the prepare methods.")
        holder._accelerator = acc
        return
    if _ACCEL["explicit"] is not None:
        raise RuntimeError("An accelerator has already been set. Make sure `train.torch.accelerate()` is not "
                           "called multiple times, and is called before any of the prepare methods.")
    _ACCEL["explicit"] = acc


def _get_accelerator() -> _Accelerator:
    """The worker's accelerator (one per Train session; a default one when ``accelerate`` was not
    called, as the reference's ``get_accelerator(_TorchAccelerator)``)."""
    from .._internal.session import _SESSION

    if _SESSION is not None:
        acc = getattr(_SESSION, "_accelerator", None)
        if acc is None:
            acc = _SESSION._accelerator = _Accelerator()
        return acc
    if _ACCEL["explicit"] is not None:
        return _ACCEL["explicit"]
    if _ACCEL["default"] is None:
        _ACCEL["default"] = _Accelerator()
    return _ACCEL["default"]


def _model_get_state(self):
    # pickling a model whose forward was replaced by an autocast wrapper: hand back the original
    # forward (and __getstate__), as the reference does
    if hasattr(self, "_original_get_state"):
        state = self._original_get_state()
        state["__getstate__"] = state["_original_get_state"]
        del state["_original_get_state"]
    else:
        state = self.__dict__.copy()
        del state["__getstate__"]
    state["forward"] = state["_unwrapped_forward"]
    del state["_unwrapped_forward"]
    return state


def _wrap_autocast(model: torch.nn.Module, acc: _Accelerator) -> torch.nn.Module:
    import functools
    import types

    if hasattr(model, "_unwrapped_forward"):
        return model
    fwd = model.forward
    device_type, dtype = acc.device_type, acc.dtype

    @functools.wraps(fwd)
    def autocast_forward(*args, **kwargs):
        with torch.autocast(device_type=device_type, dtype=dtype):
            return fwd(*args, **kwargs)

    model._unwrapped_forward = fwd
    model.forward = autocast_forward
    if hasattr(model, "__getstate__"):
        model._original_get_state = model.__getstate__
    model.__getstate__ = types.MethodType(_model_get_state, model)
    return model


def prepare_model(model: torch.nn.Module, move_to_device: bool = True, parallel_strategy: Optional[str] = "ddp",
                  parallel_strategy_kwargs: Optional[Dict[str, Any]] = None, wrap_ddp: Optional[bool] = None):
    """Move to the worker's device and wrap for data parallelism.

    ``parallel_strategy``: ``"ddp"`` (default) = the framework's bucketed RCCL DDP with flat
    gradient buckets (``ray_community_amd.parallel.DistributedDataParallel``); ``"torch_ddp"`` =
    ``torch.nn.parallel.DistributedDataParallel``; ``"fsdp"`` = torch FSDP; ``"zero3"`` = the
    framework's ZeRO-3 (``parallel.FullyShardedDataParallel``: per-block RCCL all-gather /
    reduce-scatter over flat shards; step it with ``parallel.FullyShardedAdamW`` and call
    ``finish_gradient_sync()`` after backward); ``None`` = no wrap. After ``accelerate(amp=True)``
    the model's forward runs under autocast (the parameters stay fp32).
    """
    kw = dict(parallel_strategy_kwargs or {})
    if wrap_ddp is False:
        parallel_strategy = None
    dev = move_to_device if isinstance(move_to_device, torch.device) else get_device()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if move_to_device:
        model = model.to(dev)
    acc = _get_accelerator()
    if acc.amp_is_enabled:
        model = _wrap_autocast(model, acc)
    if _world() <= 1 or parallel_strategy is None:
        return model
    if parallel_strategy == "ddp":
        from ...parallel import DistributedDataParallel

        return DistributedDataParallel(model, bucket_cap_mb=kw.pop("bucket_cap_mb", 256.0),
                                       average_in_optimizer=False, auto_finalize=True)
    if parallel_strategy == "torch_ddp":
        from torch.nn.parallel import DistributedDataParallel as TDDP

        if dev.type == "cuda":
            kw.setdefault("device_ids", [dev.index])
        return TDDP(model, **kw)
    if parallel_strategy == "zero3":
        from ...parallel import FullyShardedDataParallel

        return FullyShardedDataParallel(model, **kw)
    if parallel_strategy == "fsdp":
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP

        return FSDP(model, device_id=dev if dev.type == "cuda" else None, **kw)
    raise ValueError(f"unknown parallel_strategy {parallel_strategy}")


class _DeviceLoader:
    def __init__(self, loader, device, auto_transfer=True):
        self._loader = loader
        self.device = device
        self._auto = auto_transfer
        self.dataset = getattr(loader, "dataset", None)
        self.sampler = getattr(loader, "sampler", None)
        self.batch_size = getattr(loader, "batch_size", None)

    def _move(self, x):
        if isinstance(x, torch.Tensor):
            return x.to(self.device, non_blocking=True)
        if isinstance(x, (list, tuple)):
            return type(x)(self._move(v) for v in x)
        if isinstance(x, dict):
            return {k: self._move(v) for k, v in x.items()}
        return x

    def __len__(self):
        return len(self._loader)

    def __iter__(self):
        for b in self._loader:
            yield self._move(b) if self._auto else b


def _seeded_worker_init(seed: int, user_fn):
    def init(worker_id: int):
        import numpy as np

        ws = torch.initial_seed() % 2 ** 32
        np.random.seed(ws)
        random.seed(ws)
        if user_fn is not None:
            user_fn(worker_id)

    return init


def prepare_data_loader(data_loader, add_dist_sampler: bool = True, move_to_device: bool = True,
                        auto_transfer: bool = True):
    from torch.utils.data import DataLoader, DistributedSampler, IterableDataset, RandomSampler

    world = _world()
    seed = _get_accelerator()._seed
    if (add_dist_sampler and world > 1 and not isinstance(data_loader.dataset, IterableDataset)
            and not isinstance(data_loader.sampler, DistributedSampler)):
        import torch.distributed as dist

        shuffle = isinstance(data_loader.sampler, RandomSampler)
        sampler = DistributedSampler(data_loader.dataset, num_replicas=world, rank=dist.get_rank(), shuffle=shuffle,
                                     seed=seed if seed is not None else 0)
        wif, gen = data_loader.worker_init_fn, data_loader.generator
        if seed is not None:  # enable_reproducibility(): seeded loader workers
            wif = _seeded_worker_init(seed, wif)
            gen = torch.Generator()
            gen.manual_seed(seed)
        data_loader = DataLoader(data_loader.dataset, batch_size=data_loader.batch_size, sampler=sampler,
                                 num_workers=data_loader.num_workers, collate_fn=data_loader.collate_fn,
                                 pin_memory=data_loader.pin_memory, drop_last=data_loader.drop_last,
                                 worker_init_fn=wif, generator=gen)
    if move_to_device:
        return _DeviceLoader(data_loader, get_device(), auto_transfer)
    return data_loader


class _WrappedOptimizer(torch.optim.Optimizer):
    """``prepare_optimizer``'s result (reference ``_WrappedOptimizer``): delegates to the user's
    optimizer; with an fp16 GradScaler, ``step`` unscales, skips inf/NaN steps and updates the
    scale."""

    def __init__(self, optimizer, scaler=None):  # noqa: super().__init__ would reset param_groups
        self.optimizer = optimizer
        self.scaler = scaler

    @property
    def state(self):
        return self.optimizer.state

    @state.setter
    def state(self, state):
        self.optimizer.state = state

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @param_groups.setter
    def param_groups(self, groups):
        self.optimizer.param_groups = groups

    @property
    def defaults(self):
        return self.optimizer.defaults

    @defaults.setter
    def defaults(self, defaults):
        self.optimizer.defaults = defaults

    def add_param_group(self, param_group):
        self.optimizer.add_param_group(param_group)

    def load_state_dict(self, state_dict):
        self.optimizer.load_state_dict(state_dict)

    def state_dict(self):
        return self.optimizer.state_dict()

    def zero_grad(self, set_to_none: bool = True):
        try:
            self.optimizer.zero_grad(set_to_none=set_to_none)
        except TypeError:
            self.optimizer.zero_grad()

    def step(self, closure=None):
        if self.scaler is not None:
            self.scaler.step(self.optimizer, closure)
            self.scaler.update()
        elif closure is not None:
            return self.optimizer.step(closure)
        else:
            return self.optimizer.step()

    def __getattr__(self, name):  # FlatAdamW / FlatSGD extras (wait_pending_update, grad_scale...)
        if name in ("optimizer", "scaler"):
            raise AttributeError(name)
        return getattr(self.optimizer, name)

    def __repr__(self):
        return f"_WrappedOptimizer({self.optimizer!r}, scaler={self.scaler is not None})"


def prepare_optimizer(optimizer):
    """Wrap the optimizer for automatic mixed precision (reference
    ``train_loop_utils.py:295``): with fp16 AMP its step goes through the worker's GradScaler."""
    return _WrappedOptimizer(optimizer, _get_accelerator().scaler)


def backward(tensor: torch.Tensor):
    """``tensor.backward()``, through the GradScaler under fp16 AMP (reference ``:308``)."""
    scaler = _get_accelerator().scaler
    if scaler is not None:
        scaler.scale(tensor).backward()
    else:
        tensor.backward()


def enable_reproducibility(seed: int = 0):
    """Seed torch / Python / NumPy, disable conv autotuning, deterministic algorithms, and seed
    the data-loader workers ``prepare_data_loader`` builds (reference ``:318``)."""
    _get_accelerator()._seed = seed
    torch.manual_seed(seed)
    random.seed(seed)
    try:
        import numpy as np

        np.random.seed(seed)
    except ImportError:
        pass
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.benchmark = False


def accelerate(amp: bool = False, dtype: Optional[torch.dtype] = None):
    """Enable training optimizations (reference ``:274``): ``amp`` runs the prepared model's
    forward under autocast (bf16 by default on MI355X; ``dtype=torch.float16`` adds a GradScaler
    used by ``prepare_optimizer`` / ``backward``). Call once, before the prepare functions."""
    _set_accelerator(_Accelerator(amp=amp, dtype=dtype))


class TorchWorkerProfiler:
    """``torch.profiler`` on a Train worker (the reference's pre-2.0 API, re-enabled): use
    ``.profiler`` as the profiler context (``profiler.step()`` per iteration); each trace is
    written as chrome-trace JSON under ``trace_dir`` (default: a temp dir), named by world rank,
    and ``get_and_clear_profile_traces()`` returns the new ones as ``{"profiler_traces": [(name,
    bytes)]}`` for ``train.report``. Activities: CPU, plus the GPU (HIP through torch's CUDA
    activity) when the worker has one."""

    def __init__(self, trace_dir: Optional[str] = None, schedule=None, activities=None, **profile_kw):
        import tempfile

        from torch.profiler import ProfilerActivity, profile

        self.trace_dir = trace_dir or tempfile.mkdtemp(prefix="rca_torch_profile_")
        os.makedirs(self.trace_dir, exist_ok=True)
        self._rank = _world_rank()
        self._count = 0
        self._new = []
        if activities is None:
            activities = [ProfilerActivity.CPU]
            if torch.cuda.is_available():
                activities.append(ProfilerActivity.CUDA)
        self.profiler = profile(activities=activities, schedule=schedule, on_trace_ready=self._trace_handler,
                                **profile_kw)

    def _trace_handler(self, p):
        name = f"worker_{self._rank}_trace_{self._count}.pt.trace.json"
        self._count += 1
        path = os.path.join(self.trace_dir, name)
        p.export_chrome_trace(path)
        self._new.append(path)

    def __enter__(self):
        self.profiler.__enter__()
        return self

    def __exit__(self, *exc):
        return self.profiler.__exit__(*exc)

    def step(self):
        self.profiler.step()

    def get_and_clear_profile_traces(self):
        out = []
        for path in self._new:
            with open(path, "rb") as f:
                out.append((os.path.basename(path), f.read()))
        self._new = []
        return {"profiler_traces": out}


def _world_rank() -> int:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    try:
        from .._internal.session import _SESSION

        if _SESSION is not None:
            return int(_SESSION.context.get_world_rank())
    except Exception:
        pass
    return 0
