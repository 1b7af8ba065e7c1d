#!/bin/bash
# Round 4: hand GEMM variant 5 (partial lgkmcnt waits, no per-slice LDS drain) vs 3 vs hipBLASLt;
# numerics (all layouts, tightened bound, corrupted-K-slice check) first.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm or wgrad" > gpurun_out/r4b_tests.log 2>&1 || { tail -30 gpurun_out/r4b_tests.log; exit 1; }
tail -1 gpurun_out/r4b_tests.log
timeout -k 10 400 python -u scripts/gemm_bench.py --variants 5,3 --rounds 3 --reps 5 --json gpurun_out/r4b_gemm.json > gpurun_out/r4b_gemm.log 2>&1 || { tail -20 gpurun_out/r4b_gemm.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4b_gemm.json"))
for r in d["rows"]:
    print(f"{r['name']:11s} v5 {r['v5_tf']:7.1f}  v3 {r['v3_tf']:7.1f}  torch {r['torch_tf']:7.1f}  torch+tr {r['torch+tr_tf']:7.1f}  err5 {r['v5_err']:.1e}")
print(d["total_ms"])
PY
