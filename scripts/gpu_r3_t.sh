#!/bin/bash
# PMC passes: hand GEMM vs hipBLASLt on the o_proj wgrad product, and the attention kernels (iterative-ILP build)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 ATTN_ITERS=3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_g gpurun_out/pmc_a
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_g -o pmc --output-format csv -- python scripts/gemm_pmc_probe.py > gpurun_out/pmc_g.log 2>&1 || { echo "pmc gemm failed $?"; tail -5 gpurun_out/pmc_g.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_a -o pmc --output-format csv -- python scripts/attn_bench.py > gpurun_out/pmc_a.log 2>&1 || { echo "pmc attn failed $?"; tail -5 gpurun_out/pmc_a.log; exit 1; }
python scripts/pmc_onepass.py gpurun_out/pmc_g > gpurun_out/pmc_g_summary.md 2>&1; head -20 gpurun_out/pmc_g_summary.md
python scripts/pmc_onepass.py gpurun_out/pmc_a > gpurun_out/pmc_a_summary.md 2>&1; head -20 gpurun_out/pmc_a_summary.md
