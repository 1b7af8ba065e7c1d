#!/bin/bash
# Fused SwiGLU microbench; the step with the gate_up dgrad on the hand GEMM (variant 7) vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_swiglu_tr_gpu.py tests/test_ops_gpu.py -k "swiglu or gemm" > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -1 gpurun_out/r4i_tests.log
timeout -k 10 200 python -u scripts/swiglu_fused_bench.py > gpurun_out/r4i_swiglu.log 2>&1 || { tail -20 gpurun_out/r4i_swiglu.log; exit 1; }
cat gpurun_out/r4i_swiglu.log
for i in 1 2; do
RCA_DGRAD_PLAN=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4i_bench_plan$i.log 2>&1 || { tail -20 gpurun_out/r4i_bench_plan$i.log; exit 1; }
tail -1 gpurun_out/r4i_bench_plan$i.log | cut -c1-160
RCA_DGRAD_PLAN=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4i_bench_noplan$i.log 2>&1 || { tail -20 gpurun_out/r4i_bench_noplan$i.log; exit 1; }
tail -1 gpurun_out/r4i_bench_noplan$i.log | cut -c1-160
done
