#!/bin/bash
# in-process kernel profile of the 8B training step (rocprofv3 kernel trace + stats)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof8b
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python scripts/prof_llama.py --steps 3 > gpurun_out/prof8b.log 2>&1 && echo "prof ok" || exit 1
grep "ms/step" gpurun_out/prof8b.log
python scripts/rocpd_summary.py $(find gpurun_out/prof8b -name "*.db" | head -1) 40 > gpurun_out/prof8b_summary.md
head -30 gpurun_out/prof8b_summary.md
