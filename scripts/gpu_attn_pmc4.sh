#!/bin/bash
# hand-scheduled attention forward (RCA_ATTN_FWD=hs) vs the default: SQ cycle breakdown and MFMA /
# VALU / LDS activity -- one --pmc pass each (8 SQ counters + GRBM_GUI_ACTIVE), kernel trace only
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for mode in hs narrow; do
  RCA_ATTN_FWD=$mode timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_attn4_$mode -o pmc --output-format csv \
    -- python scripts/attn_bench.py > gpurun_out/pmc_attn4_$mode.log 2>&1 || exit 1
done
