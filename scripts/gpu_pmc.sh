#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_kernels.py (one counter group per run, kernel trace only):
#   A: SQ occupancy/stall/LDS/MFMA counters + GRBM_GUI_ACTIVE  B: FETCH_SIZE  C: WRITE_SIZE
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/a -o run --output-format csv -- python scripts/pmc_kernels.py > gpurun_out/pmc_a.log 2>&1 || { echo "pass A failed"; tail -5 gpurun_out/pmc_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc/b -o run --output-format csv -- python scripts/pmc_kernels.py > gpurun_out/pmc_b.log 2>&1 || { echo "pass B failed"; tail -5 gpurun_out/pmc_b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc/c -o run --output-format csv -- python scripts/pmc_kernels.py > gpurun_out/pmc_c.log 2>&1 || { echo "pass C failed"; tail -5 gpurun_out/pmc_c.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.md && cat gpurun_out/pmc_summary.md
