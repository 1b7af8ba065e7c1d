#!/bin/bash
# flash-attention numerics + microbenchmark
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -q --timeout 200 > gpurun_out/pytest_attn.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -25 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; echo "bench exit $?"; grep -v amdgpu.ids gpurun_out/attn_bench.log
