#!/bin/bash
# PMC passes on the k-contiguous o_proj forward GEMM: hand variants 6 / 3 vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_d1 gpurun_out/pmc_d2 gpurun_out/pmc_d3
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r4d_avail.txt 2>&1 || echo "list-avail rc $?"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace -d gpurun_out/pmc_d1 -o pmc --output-format csv -- python scripts/gemm_pmc_tn.py > gpurun_out/pmc_d1.log 2>&1 || { echo "pmc d1 failed $?"; tail -5 gpurun_out/pmc_d1.log; exit 1; }
python scripts/pmc_onepass.py gpurun_out/pmc_d1 > gpurun_out/pmc_d1_summary.md 2>&1; head -8 gpurun_out/pmc_d1_summary.md
C2="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C2 --kernel-trace -d gpurun_out/pmc_d2 -o pmc --output-format csv -- python scripts/gemm_pmc_tn.py > gpurun_out/pmc_d2.log 2>&1 || { echo "pmc d2 failed $?"; tail -5 gpurun_out/pmc_d2.log; exit 1; }
python - > gpurun_out/pmc_d2_summary.md 2>&1 <<'PY'
import sys
sys.path.insert(0, "scripts")
from pmc_summary import load, short
A = load("gpurun_out/pmc_d2")
for k in sorted(A, key=lambda k: -A[k]["_t"]):
    a = A[k]
    n = a["_n"]
    print(short(k, 60), f"n={int(n)} us={a['_t'] / n * 1e6:.1f}", " ".join(f"{c}={v / n:.4g}" for c, v in sorted(a.items()) if not c.startswith("_")))
PY
head -20 gpurun_out/pmc_d2_summary.md
