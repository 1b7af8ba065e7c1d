#!/bin/bash
# Round 2, session 2 first call: full GPU suite, smoke, headline bench (N=1), kernel profile of the 8B step.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_d.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu_d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_d.log 2>&1 && tail -1 gpurun_out/bench_d.log || exit 1
bash scripts/gpu_prof8b.sh
