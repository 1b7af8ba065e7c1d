#!/bin/bash
# after the core transport fixes (GIL-free blocked sends, log forwarding): GPU suite + smoke +
# headline bench + the secondary BASELINE configs (ResNet-50, RLlib PPO, Data->Serve)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench.log 2>/dev/null || exit 1
echo "bench stdout lines: $(wc -l < gpurun_out/bench.log)"; tail -1 gpurun_out/bench.log
timeout -k 10 400 python bench_resnet.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1; echo "resnet rc $?"; tail -1 gpurun_out/bench_resnet.log
timeout -k 10 400 python bench_rllib.py --learners 1 --iters 5 --warmup 1 > gpurun_out/bench_rllib.log 2>&1; echo "rllib rc $?"; tail -1 gpurun_out/bench_rllib.log
timeout -k 10 400 python bench_data_serve.py --gpus 1 --batches 20 --warmup 3 > gpurun_out/bench_data_serve.log 2>&1; echo "data_serve rc $?"; tail -1 gpurun_out/bench_data_serve.log
