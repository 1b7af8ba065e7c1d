#!/bin/bash
# GPU object layout fix: runtime tests + data->serve diag + bench
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_j.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag/data_serve_diag.py > gpurun_out/ds_diag.log 2>&1; echo "diag rc $?"; tail -3 gpurun_out/ds_diag.log
timeout -k 10 400 python bench_data_serve.py --gpus 1 --batches 20 --warmup 3 > gpurun_out/bench_data_serve.log 2>&1; echo "data_serve rc $?"; tail -1 gpurun_out/bench_data_serve.log
