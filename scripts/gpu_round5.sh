#!/bin/bash
# GPU tests + smoke + bench + in-process kernel profile of the 8B training step.
# Every GPU step has its own time limit; steps are chained so the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run -- python scripts/prof_llama.py --steps 3 > gpurun_out/prof8b.log 2>&1 && echo "prof ok" || exit 1
grep "ms/step" gpurun_out/prof8b.log
find gpurun_out/prof8b -name "*stats*"
