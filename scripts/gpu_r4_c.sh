#!/bin/bash
# Round 4: hand GEMM variant 6 (buffer-descriptor LDS-DMA, immediate-offset fragment reads, no
# vector address arithmetic in the loop) vs variant 3 vs hipBLASLt, on natural and TN layouts.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm or wgrad" > gpurun_out/r4c_tests.log 2>&1 || { tail -30 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
timeout -k 10 500 python -u scripts/gemm_bench.py --variants 6,3 --tn --rounds 3 --reps 5 --json gpurun_out/r4c_gemm.json > gpurun_out/r4c_gemm.log 2>&1 || { tail -20 gpurun_out/r4c_gemm.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4c_gemm.json"))
for r in d["rows"]:
    print(f"{r['name']:11s} v6tn {r['v6_tn_tf']:7.1f} v3tn {r['v3_tn_tf']:7.1f} torch_tn {r['torch_tn_tf']:7.1f} | nat v6 {r['v6_tf']:7.1f} v3 {r['v3_tf']:7.1f} torch {r['torch_tf']:7.1f} torch+tr {r['torch+tr_tf']:7.1f} err6tn {r['v6_tn_err']:.1e}")
print(d["total_ms"])
PY
