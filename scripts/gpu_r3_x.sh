#!/bin/bash
# GBDT histogram kernel: packed fixed-point u64 LDS atomics; tests, bench, one PMC pass on the kernel alone
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
timeout -k 10 300 python -u scripts/gbdt_bench.py > gpurun_out/r3x_bench.log 2>&1 && timeout -k 10 300 python -u scripts/gbdt_bench.py --rows 10500000 --rounds 50 >> gpurun_out/r3x_bench.log 2>&1 || { tail -30 gpurun_out/r3x_bench.log; exit 1; }
grep metric gpurun_out/r3x_bench.log
rm -rf gpurun_out/pmc_gbx
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_gbx -o pmc --output-format csv -- python scripts/gbdt_bench.py --hist-only > gpurun_out/pmc_gbx.log 2>&1 || { echo "pmc failed $?"; tail -5 gpurun_out/pmc_gbx.log; exit 1; }
python scripts/pmc_onepass.py gpurun_out/pmc_gbx > gpurun_out/pmc_gbx_summary.md 2>&1; head -8 gpurun_out/pmc_gbx_summary.md
