"""Build the native runtime core (``_rca_native``: shm object store + scheduler) in-tree with g++."""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB_PATH = os.path.join(HERE, "_rca_native" + EXT)


def _sources():
    return sorted(glob.glob(os.path.join(HERE, "*.cpp")))


def _digest():
    h = hashlib.sha256()
    for p in _sources():
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def is_stale():
    stamp = LIB_PATH + ".stamp"
    if not os.path.exists(LIB_PATH) or not os.path.exists(stamp):
        return True
    return open(stamp).read().strip() != _digest()


def build(force=False, verbose=False):
    if not force and not is_stale():
        return LIB_PATH
    import pybind11

    inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
    tmp = LIB_PATH + f".tmp{os.getpid()}"
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]
    cmd += [f"-I{i}" for i in inc] + _sources() + ["-o", tmp, "-lpthread", "-lrt"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + r.stdout + r.stderr)
    os.replace(tmp, LIB_PATH)
    with open(LIB_PATH + ".stamp", "w") as f:
        f.write(_digest())
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
