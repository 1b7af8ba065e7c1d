#!/bin/bash
# secondary BASELINE configs on round-4 code: ResNet-50 DDP, RLlib PPO Atari, Data -> Serve
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench_resnet.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4s_resnet.json 2> gpurun_out/r4s_resnet.err || { tail -20 gpurun_out/r4s_resnet.err; exit 1; }
tail -1 gpurun_out/r4s_resnet.json
timeout -k 10 400 python -u bench_rllib.py --learners 1 --iters 5 --warmup 1 > gpurun_out/r4s_rllib.json 2> gpurun_out/r4s_rllib.err || { tail -20 gpurun_out/r4s_rllib.err; exit 1; }
tail -1 gpurun_out/r4s_rllib.json
timeout -k 10 400 python -u bench_data_serve.py --gpus 1 --batches 40 --warmup 6 > gpurun_out/r4s_data_serve.json 2> gpurun_out/r4s_data_serve.err || { tail -20 gpurun_out/r4s_data_serve.err; exit 1; }
tail -1 gpurun_out/r4s_data_serve.json
