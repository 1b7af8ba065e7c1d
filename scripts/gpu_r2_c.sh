#!/bin/bash
# Round 2, call C: full GPU suite (GEMM numerics, GPU object store spill/restore + owner death,
# direct actor transport on GPU actors), smoke, headline bench self-launched (N=1).
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu_c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_c.log 2>&1 && tail -1 gpurun_out/bench_c.log || exit 1
