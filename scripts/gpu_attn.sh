#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; echo "attn exit $?"; cat gpurun_out/attn_bench.log | grep -v amdgpu.ids
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -k rmsnorm > gpurun_out/pytest_rms.log 2>&1; echo "pytest exit $?"; tail -2 gpurun_out/pytest_rms.log
