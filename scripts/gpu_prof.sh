#!/bin/bash
# kernel-level profile of the 8B bench + GPU tests
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
env | grep -i -E "visible|rocr|hip_" > gpurun_out/env.txt
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof8b.log 2>&1; echo "prof exit $?"
tail -2 gpurun_out/prof8b.log
find gpurun_out/prof8b -name "*stats*" | head
