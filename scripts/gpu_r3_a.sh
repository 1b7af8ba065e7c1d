#!/bin/bash
# round 3: ping-pong GEMM numerics + A/B vs round-2 variant and hipBLASLt on the 8B shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k gemm > gpurun_out/r3a_test.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/r3a_test.log; exit 1; }
tail -3 gpurun_out/r3a_test.log
timeout -k 10 400 python -u scripts/gemm_bench.py --rounds 3 --reps 5 --variants 2,0 --json gpurun_out/r3a_gemm.json > gpurun_out/r3a_gemm.log 2>&1
rc=$?
cat gpurun_out/r3a_gemm.log
exit $rc
