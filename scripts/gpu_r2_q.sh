#!/bin/bash
# attention hazard fix: determinism diag + attention tests + attention microbench + full GPU suite + bench
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONPATH=$PWD
timeout -k 10 200 python -u scripts/diag/fwd_det.py > gpurun_out/q_fwd.log 2>&1; rc=$?; tail -9 gpurun_out/q_fwd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/q_attn_bench.log 2>&1 || { tail gpurun_out/q_attn_bench.log; exit 1; }
grep rca-hip gpurun_out/q_attn_bench.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
