#!/bin/bash
# gemm4 slice ring (3) vs two-stage (2) vs hipBLASLt: numerics on all layouts, then timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k gemm > gpurun_out/r3d_test.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/r3d_test.log; exit 1; }
tail -2 gpurun_out/r3d_test.log
timeout -k 10 400 python -u scripts/gemm_bench.py --rounds 3 --reps 5 --variants 3,2 --json gpurun_out/r3d_gemm.json > gpurun_out/r3d_gemm.log 2>&1
rc=$?
python3 - <<'PY'
import json
for l in open('gpurun_out/r3d_gemm.log'):
    if l.startswith('{"name'):
        r=json.loads(l); print(r['name'], r['v3_err'], r['v3_acc_err'], r['v3_tf'], r['v2_tf'], r['torch_tf'], r['torch+tr_tf'])
    elif 'total' in l: print(l.strip())
PY
exit $rc
