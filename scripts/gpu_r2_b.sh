#!/bin/bash
# Round 2, call B: overlapped-AdamW correctness test, then the headline bench with the update
# overlapped with the next forward (default) vs serial.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "overlapped or adamw" > gpurun_out/pytest_b.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_ov.log 2>&1 && tail -1 gpurun_out/bench_ov.log || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 --no-overlap-optimizer > gpurun_out/bench_serial.log 2>&1 && tail -1 gpurun_out/bench_serial.log || exit 1
