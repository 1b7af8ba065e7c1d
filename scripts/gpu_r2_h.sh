#!/bin/bash
# transposed SwiGLU outputs: tests + bench + kernel profile
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_swiglu_tr_gpu.py tests/test_ops_gpu.py tests/test_fused_ce_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_h.log 2>&1 && tail -1 gpurun_out/bench_h.log || exit 1
bash scripts/gpu_prof8b.sh
