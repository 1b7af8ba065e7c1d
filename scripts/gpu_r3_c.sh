#!/bin/bash
# gemm4 register-staged: numerics (all layouts) + A/B vs no-global-load diagnostic and hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k gemm > gpurun_out/r3c_test.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/r3c_test.log; exit 1; }
tail -2 gpurun_out/r3c_test.log
timeout -k 10 400 python -u scripts/gemm_bench.py --rounds 3 --reps 5 --variants 2,91,92 --only wgrad --json gpurun_out/r3c_gemm.json > gpurun_out/r3c_gemm.log 2>&1
rc=$?
cat gpurun_out/r3c_gemm.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{\"name'):
        r=json.loads(l); print(r['name'], r['v2_err'], r['v2_acc_err'], r['v2_tf'], r["v91_tf"], r["v92_tf"], r['torch_tf'], r['torch+tr_tf'])
    elif 'total' in l: print(l.strip())
"
exit $rc
