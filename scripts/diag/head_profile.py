"""cProfile of the head's event-loop thread while one core-microbenchmark row runs.

    python scripts/diag/head_profile.py "multi client tasks async"
"""
import cProfile
import pstats
import sys

sys.path.insert(0, ".")
from ray_community_amd._private import head as H  # noqa: E402
from ray_community_amd._private import ray_perf  # noqa: E402

prof = cProfile.Profile()
_orig = H.Head._loop


def _loop(self):
    prof.enable()
    try:
        _orig(self)
    finally:
        prof.disable()


H.Head._loop = _loop
ray_perf.run(window=2.0, rounds=2, pattern=sys.argv[1] if len(sys.argv) > 1 else "multi client tasks async")
st = pstats.Stats(prof)
st.sort_stats("tottime").print_stats(30)
