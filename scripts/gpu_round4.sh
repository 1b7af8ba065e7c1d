#!/bin/bash
# GPU tests + in-process kernel profile of the 8B training step
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"; tail -4 gpurun_out/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python scripts/prof_llama.py --steps 3 > gpurun_out/prof8b.log 2>&1 && echo "prof ok"
grep "ms/step" gpurun_out/prof8b.log
find gpurun_out/prof8b -name "*.db" -o -name "*stats*" | head
