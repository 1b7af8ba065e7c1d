#!/bin/bash
# RMSNorm backward rewrite: numerics (GPU op tests), then new vs old library timing.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_ops.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/rms_bench.py > gpurun_out/rms_new.log 2>&1 && tail -1 gpurun_out/rms_new.log || exit 1
RCA_KERNEL_LIB=$PWD/abtest/libraca_old.so timeout -k 10 120 python scripts/rms_bench.py > gpurun_out/rms_old.log 2>&1 && tail -1 gpurun_out/rms_old.log || exit 1
timeout -k 10 120 env H=2048 python scripts/rms_bench.py 2>&1 | tail -1
