#!/bin/bash
# Re-check after the GC tuning commit: GPU tests, smoke, headline bench (DDP) and the ZeRO path
# the N>1 runs take, both at N=1. Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --parallel zero > gpurun_out/bench_zero1.log 2>&1 && tail -1 gpurun_out/bench_zero1.log || exit 1
