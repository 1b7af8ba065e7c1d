#!/bin/bash
# sumsq kernel with 4 loads in flight per lane: microbench + numerics, DDP norm tests, bench
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONPATH=$PWD
timeout -k 10 120 python scripts/sumsq_bench.py > gpurun_out/u_sumsq.log 2>&1; rc=$?; tail -2 gpurun_out/u_sumsq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ddp_norm_gpu.py tests/test_ops_gpu.py > gpurun_out/u_tests.log 2>&1; rc=$?; tail -2 gpurun_out/u_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/u_bench.log 2>/dev/null || exit 1
tail -1 gpurun_out/u_bench.log
