#!/bin/bash
# per-kernel time + SQ counters for the attention kernels
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
export ATTN_ITERS=3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run -- python scripts/attn_bench.py > gpurun_out/prof_attn.log 2>&1; echo "trace exit $?"
python scripts/rocpd_summary.py $(find gpurun_out/prof_attn -name "*.db" | head -1) 8
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc_attn -o pmc --output-format csv -- python scripts/attn_bench.py > gpurun_out/pmc_attn.log 2>&1; echo "pmc exit $?"
find gpurun_out/pmc_attn -name "*counter_collection*" | head -3
