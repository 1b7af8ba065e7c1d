#!/bin/bash
# transpose kernel numerics + backward-GEMM layout A/B inside the full 8B step
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "transpose or fused_wgrad or llama" > gpurun_out/pytest_tr.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_tr.log
[ $rc -eq 0 ] || exit $rc
RCA_BWD_TRANSPOSED=0 timeout -k 10 300 python scripts/prof_llama.py --steps 5 > gpurun_out/step_tr0.log 2>&1 || { tail -20 gpurun_out/step_tr0.log; exit 1; }
grep "ms/step" gpurun_out/step_tr0.log
RCA_BWD_TRANSPOSED=1 timeout -k 10 300 python scripts/prof_llama.py --steps 5 > gpurun_out/step_tr1.log 2>&1 || { tail -20 gpurun_out/step_tr1.log; exit 1; }
grep "ms/step" gpurun_out/step_tr1.log
