#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"; tail -15 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_8b.log 2>&1; echo "bench exit $?"; grep -v amdgpu.ids gpurun_out/bench_8b.log | tail -3
