#!/bin/bash
# ZeRO-3 GPU test + PMC passes
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_fully_sharded.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fsdp.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fsdp.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh
