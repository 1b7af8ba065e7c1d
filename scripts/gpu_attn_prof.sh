#!/bin/bash
# kernel-level timing of the attention kernels at the 8B bench shape
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run -- python scripts/attn_bench.py > gpurun_out/prof_attn.log 2>&1; echo "prof exit $?"
grep -v amdgpu.ids gpurun_out/prof_attn.log | grep -E "rca-hip|sdpa"
python scripts/rocpd_summary.py $(find gpurun_out/prof_attn -name "*.db" | head -1) 12
