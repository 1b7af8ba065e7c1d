#!/bin/bash
# attention kernels: SQ cycle breakdown (wave cycles = wait + wait_inst + active), MFMA busy,
# LDS conflict / active cycles -- one pass of 8 SQ counters + GRBM_GUI_ACTIVE
set -o pipefail
mkdir -p gpurun_out
export ATTN_ITERS=3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_attn3 -o pmc --output-format csv -- python scripts/attn_bench.py > gpurun_out/pmc_attn3.log 2>&1; echo "pmc exit $?"
tail -3 gpurun_out/pmc_attn3.log
