#!/bin/bash
# secondary BASELINE configs on 1 GPU: ResNet-50 DDP, RLlib PPO (1 GPU learner), Data->Serve pipeline
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 400 python bench_resnet.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1; echo "resnet rc $?"; tail -1 gpurun_out/bench_resnet.log
timeout -k 10 400 python bench_rllib.py --learners 1 --iters 5 --warmup 1 > gpurun_out/bench_rllib.log 2>&1; echo "rllib rc $?"; tail -1 gpurun_out/bench_rllib.log
timeout -k 10 400 python bench_data_serve.py --gpus 1 --batches 20 --warmup 3 > gpurun_out/bench_data_serve.log 2>&1; echo "data_serve rc $?"; tail -1 gpurun_out/bench_data_serve.log
