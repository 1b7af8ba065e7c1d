#!/bin/bash
# dK/dV: compile-time diagonal variant + dP initialised with -delta
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/attn_bench_l.log
