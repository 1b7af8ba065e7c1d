#!/bin/bash
# ResNet-50 + RLlib benches, kernel tests, ResNet kernel profile. Each GPU step time-limited; first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "batch_norm or resnet or image" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_ops.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench_resnet.py --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1 && tail -1 gpurun_out/bench_resnet.log || { tail -20 gpurun_out/bench_resnet.log; exit 1; }
timeout -k 10 400 python bench_rllib.py > gpurun_out/bench_rllib.log 2>&1 && tail -1 gpurun_out/bench_rllib.log || { tail -20 gpurun_out/bench_rllib.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profrn -o run -- python scripts/prof_resnet.py --steps 5 > gpurun_out/profrn.log 2>&1 && echo "prof ok" && grep "ms/step" gpurun_out/profrn.log
