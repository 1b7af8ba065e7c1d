"""Build the gfx950 HIP kernel library (``libraca_kernels.so``) in-tree.

The kernels expose a plain C ABI (``extern "C" rca_*``) taking raw device pointers and a
``hipStream_t``; Python binds them with ctypes (``ops/_lib.py``). No torch C++ headers, no
hipify, no CUDA shims: ``hipcc --offload-arch=gfx950`` on the ``.hip`` sources only.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_NAME = "libraca_kernels.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
ARCH = os.environ.get("RCA_OFFLOAD_ARCH", "gfx950")
# Keep loop-carried MFMA accumulators in the accumulator file: without this hipcc copies every
# AGPR-resident accumulator to VGPRs and back around each loop iteration once a kernel's live set
# exceeds 256 VGPRs (the one-wave-per-SIMD attention dK/dV kernel: 574 v_accvgpr moves -> 26).
EXTRA_FLAGS = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
# per-file overrides: the one-wave-per-SIMD kernels (dK/dV, the 4-wave GEMM) keep their
# accumulators in AGPRs. The attention kernels use LLVM's iterative-ILP machine-scheduling
# strategy: fwd+bwd 1.489 vs 1.512 ms at the 8B shape over three interleaved rounds (max-ilp,
# max-memory-clause and iterative-minreg were 2-8 % slower; scripts/ab_sched_build.sh,
# scripts/gpu_r3_q.sh, profiles/attn_sched_r3.log).
_ILP = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
FILE_FLAGS = {"attention_dkdv.hip": _ILP, "attention_fwd_wide.hip": _ILP, "attention_fwd_hs.hip": _ILP, "gemm4.hip": [],
              "attention.hip": EXTRA_FLAGS + _ILP}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the gfx950 kernels)")


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _digest() -> str:
    h = hashlib.sha256()
    for p in _sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode())
            h.update(f.read())
    h.update(ARCH.encode())
    h.update(" ".join(EXTRA_FLAGS).encode())
    h.update(repr(sorted(FILE_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def is_stale() -> bool:
    stamp = LIB_PATH + ".stamp"
    if not os.path.exists(LIB_PATH) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not is_stale():
        return LIB_PATH
    objs = []
    hipcc = _hipcc()
    tmpdir = os.path.join(HERE, "_build")
    os.makedirs(tmpdir, exist_ok=True)
    procs = []
    for src in _sources():
        obj = os.path.join(tmpdir, os.path.basename(src) + ".o")
        flags = FILE_FLAGS.get(os.path.basename(src), EXTRA_FLAGS)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj] + flags
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), src))
        objs.append(obj)
    for p, src in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{out.decode(errors='replace')}")
    tmp_lib = LIB_PATH + f".tmp{os.getpid()}"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_lib] + objs
    r = subprocess.run(cmd, capture_output=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout.decode()}{r.stderr.decode()}")
    # resolve every symbol now (ctypes dlopens with RTLD_NOW): a kernel template whose host stub
    # hipcc did not emit fails here, at build time, instead of at first use on a GPU box
    import ctypes

    try:
        ctypes.CDLL(tmp_lib)
    except OSError as e:
        raise RuntimeError(f"built library does not load: {e}") from None
    os.replace(tmp_lib, LIB_PATH)
    with open(LIB_PATH + ".stamp", "w") as f:
        f.write(_digest())
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
