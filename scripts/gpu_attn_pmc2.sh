#!/bin/bash
# PMC pass over the attention microbenchmark (one counter group per run)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 ATTN_ITERS=2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_attn
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc_attn -o run --output-format csv -- python scripts/attn_bench.py > gpurun_out/pmc_attn.log 2>&1; echo "rc $?"
find gpurun_out/pmc_attn -name "*counter_collection*" | head
