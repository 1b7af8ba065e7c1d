#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"; tail -6 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench_rllib.py --iters 3 > gpurun_out/bench_rllib.log 2>&1; echo "rllib exit $?"; grep -v amdgpu.ids gpurun_out/bench_rllib.log | tail -2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8b -o run -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof8b.log 2>&1; echo "prof exit $?"
ls gpurun_out/prof8b | head
