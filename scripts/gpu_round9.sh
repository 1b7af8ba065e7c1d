#!/bin/bash
# attention kernel split + 1-GPU bench + in-process kernel profile of the 8B step
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run -- python scripts/attn_bench.py > gpurun_out/prof_attn.log 2>&1 || { tail -20 gpurun_out/prof_attn.log; exit 1; }
grep -E "rca-hip|sdpa" gpurun_out/prof_attn.log
python scripts/rocpd_summary.py $(find gpurun_out/prof_attn -name "*.db" | head -1) 8
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python scripts/prof_llama.py --steps 3 > gpurun_out/prof8b.log 2>&1 && echo "prof ok" || exit 1
grep "ms/step" gpurun_out/prof8b.log
python scripts/rocpd_summary.py $(find gpurun_out/prof8b -name "*.db" | head -1) 30 > gpurun_out/prof8b_summary.md
head -16 gpurun_out/prof8b_summary.md
