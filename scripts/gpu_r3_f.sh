#!/bin/bash
# split-master AdamW: GPU numerics tests, kernel A/B on the 8B parameter count, the 8B bench;
# aux (image / RL) kernels under rocprofv3 --stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "adamw" tests/test_telemetry.py tests/test_gpu_runtime.py::test_ppo_lstm_gpu_learner \
  > gpurun_out/r3g_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3g_tests.log; exit 1; }
tail -3 gpurun_out/r3g_tests.log
timeout -k 10 200 python -u scripts/adamw_bench.py > gpurun_out/r3g_adamw.json 2> gpurun_out/r3g_adamw.err || { echo adamw bench failed; tail gpurun_out/r3g_adamw.err; exit 1; }
cat gpurun_out/r3g_adamw.json
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3g_bench.json 2> gpurun_out/r3g_bench.err || { echo bench failed; tail gpurun_out/r3g_bench.err; exit 1; }
cat gpurun_out/r3g_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_aux -o aux -- python -u scripts/aux_kernels_bench.py \
  > gpurun_out/r3g_aux.log 2>&1 || { echo aux failed; tail gpurun_out/r3g_aux.log; exit 1; }
grep '"op"' gpurun_out/r3g_aux.log
echo exit=0
