#!/bin/bash
# PMC passes on the k-contiguous o_proj forward GEMM: hand variants 6 / 3 vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_f1 gpurun_out/pmc_f2 gpurun_out/pmc_f3
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace -d gpurun_out/pmc_f1 -o pmc --output-format csv -- python scripts/gemm_pmc_tn.py > gpurun_out/pmc_f1.log 2>&1 || { echo "pmc d1 failed $?"; tail -5 gpurun_out/pmc_f1.log; exit 1; }
python scripts/pmc_onepass.py gpurun_out/pmc_f1 > gpurun_out/pmc_f1_summary.md 2>&1; head -8 gpurun_out/pmc_f1_summary.md
C2="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $C2 --kernel-trace -d gpurun_out/pmc_f2 -o pmc --output-format csv -- python scripts/gemm_pmc_tn.py > gpurun_out/pmc_f2.log 2>&1 || { echo "pmc d2 failed $?"; tail -5 gpurun_out/pmc_f2.log; exit 1; }
python - > gpurun_out/pmc_f2_summary.md 2>&1 <<'PY'
import sys
sys.path.insert(0, "scripts")
from pmc_summary import load, short
A = load("gpurun_out/pmc_f2")
for k in sorted(A, key=lambda k: -A[k]["_t"]):
    a = A[k]
    n = a["_n"]
    print(short(k, 60), f"n={int(n)} us={a['_t'] / n * 1e6:.1f}", " ".join(f"{c}={v / n:.4g}" for c, v in sorted(a.items()) if not c.startswith("_")))
PY
head -20 gpurun_out/pmc_f2_summary.md
C3="SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_WAVE_CYCLES TA_ADDR_STALLED_BY_TD_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C3 --kernel-trace -d gpurun_out/pmc_f3 -o pmc --output-format csv -- python scripts/gemm_pmc_tn.py > gpurun_out/pmc_f3.log 2>&1 || { echo "pmc f3 failed $?"; tail -5 gpurun_out/pmc_f3.log; exit 1; }
python - > gpurun_out/pmc_f3_summary.md 2>&1 <<'PY'
import sys
sys.path.insert(0, "scripts")
from pmc_summary import load, short
A = load("gpurun_out/pmc_f3")
for k in sorted(A, key=lambda k: -A[k]["_t"]):
    a = A[k]
    n = a["_n"]
    print(short(k, 60), f"n={int(n)} us={a['_t'] / n * 1e6:.1f}", " ".join(f"{c}={v / n:.4g}" for c, v in sorted(a.items()) if not c.startswith("_")))
PY
head -20 gpurun_out/pmc_f3_summary.md
