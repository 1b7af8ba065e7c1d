#!/bin/bash
# the non-default data-parallel modes of the headline bench at full 8B scale on one GPU:
# ZeRO-1/2 (sharded AdamW), ZeRO-3 (per-block all-gather of sharded weights), fp32 gradient reduce
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
for mode in zero fsdp; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 6 --warmup 2 --parallel $mode > gpurun_out/v_$mode.log 2>&1 || { tail -20 gpurun_out/v_$mode.log; exit 1; }
  echo "$mode: $(tail -1 gpurun_out/v_$mode.log | cut -c1-330)"
done
timeout -k 10 500 python bench.py --gpus 1 --steps 6 --warmup 2 --grad-reduce-dtype fp32 > gpurun_out/v_fp32.log 2>&1 || { tail -20 gpurun_out/v_fp32.log; exit 1; }
echo "ddp fp32-reduce: $(tail -1 gpurun_out/v_fp32.log | cut -c1-330)"
