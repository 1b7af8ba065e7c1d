#!/bin/bash
# fused CE + ZeRO-3 GPU tests, PMC passes, bench A/B of the fused CE path
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_fully_sharded.py tests/test_fused_ce_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 --fused-ce 1 > gpurun_out/bench_fce.log 2>&1 && tail -1 gpurun_out/bench_fce.log || exit 1
bash scripts/gpu_pmc.sh
