#!/bin/bash
# AdamW ulp diagnostic, telemetry capture + GPU telemetry / LSTM tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/diag/adamw_ulp.py > gpurun_out/adamw_ulp.log 2>&1 || { echo "diag failed"; tail gpurun_out/adamw_ulp.log; exit 1; }
tail -8 gpurun_out/adamw_ulp.log
bash scripts/capture_telemetry.sh
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_telemetry.py tests/test_gpu_runtime.py -k "hbm_gauge or lstm" > gpurun_out/r3h_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r3h_tests.log
echo exit=$rc
