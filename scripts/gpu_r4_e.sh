#!/bin/bash
# Round 4: hand GEMM variant 7 (64-deep tiles, full-line DMA) vs 6 vs hipBLASLt.
# vector address arithmetic in the loop) vs variant 3 vs hipBLASLt, on natural and TN layouts.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm or wgrad" > gpurun_out/r4e_tests.log 2>&1 || { tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -1 gpurun_out/r4e_tests.log
timeout -k 10 500 python -u scripts/gemm_bench.py --variants 7,6 --tn --rounds 3 --reps 5 --json gpurun_out/r4e_gemm.json > gpurun_out/r4e_gemm.log 2>&1 || { tail -20 gpurun_out/r4e_gemm.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4e_gemm.json"))
for r in d["rows"]:
    print(f"{r['name']:11s} v7tn {r['v7_tn_tf']:7.1f} v6tn {r['v6_tn_tf']:7.1f} torch_tn {r['torch_tn_tf']:7.1f} | nat v7 {r['v7_tf']:7.1f} v6 {r['v6_tf']:7.1f} torch {r['torch_tf']:7.1f} torch+tr {r['torch+tr_tf']:7.1f} err7tn {r['v7_tn_err']:.1e}")
print(d["total_ms"])
PY
