#!/bin/bash
# Full GPU tier after the round-1 perf + API work: GPU tests, smoke, headline bench, RLlib PPO and
# ResNet-50 benches. Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
timeout -k 10 400 python bench_rllib.py --iters 5 --warmup 1 > gpurun_out/bench_rllib.log 2>&1 && tail -1 gpurun_out/bench_rllib.log || { tail -20 gpurun_out/bench_rllib.log; exit 1; }
timeout -k 10 400 python bench_resnet.py > gpurun_out/bench_resnet.log 2>&1 && tail -1 gpurun_out/bench_resnet.log || { tail -20 gpurun_out/bench_resnet.log; exit 1; }
