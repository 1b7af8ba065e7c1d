#!/usr/bin/env python3
"""Core-runtime microbenchmark (BASELINE.json config "Ray Core microbenchmark (tasks/sec + actor
calls/sec) local CPU-only"): same workloads and row names as the reference's ``ray microbenchmark``
(``python/ray/_private/ray_perf.py``), compared row by row with its published
``release/release_logs/2.9.3/microbenchmark.json``.

    python bench_core.py [--mode colocated|separate|both] [--window 2] [--rounds 4] [--filter PATTERN]
                         [--out profiles/core_microbenchmark.json]

``--mode separate`` runs the driver as its own process against a head started by the CLI
(``ray.init(address="auto")``); ``both`` runs the two back to back (``--out`` gets a ``_MODE``
suffix per mode).

Prints one line per row, then ONE JSON summary line (geometric mean of value / reference).
"""
import argparse
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=float, default=2.0, help="seconds per timed round")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--filter", default="")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--mode", default="colocated", choices=["colocated", "separate", "both"])
    a = ap.parse_args()
    from ray_community_amd._private import ray_perf

    modes = ["colocated", "separate"] if a.mode == "both" else [a.mode]
    for mode in modes:
        out = a.out
        if out and a.mode == "both":
            root, ext = os.path.splitext(out)
            out = f"{root}_{mode}{ext}"
        results = ray_perf.run(window=a.window, rounds=a.rounds, pattern=a.filter, scale=a.scale, mode=mode)
        doc = ray_perf.report(results, out, mode=mode)
        ratios = [r["vs_reference"] for r in doc["results"].values() if r["vs_reference"]]
        geo = math.exp(sum(math.log(x) for x in ratios) / len(ratios)) if ratios else None
        print(json.dumps({"metric": "ray_core_microbenchmark_geomean_vs_reference", "mode": mode,
                          "value": round(geo, 3) if geo else None, "unit": "x reference", "rows": len(ratios),
                          "higher_is_better": True, "cpus": doc["cpus"], "reference_hw": doc["reference_hw"]}),
              flush=True)


if __name__ == "__main__":
    main()
