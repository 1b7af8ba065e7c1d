#!/bin/bash
# Build A/B kernel libraries where attention.hip + attention_dkdv.hip use a different AMDGPU
# machine-scheduler strategy (scripts/ab_lib/libraca_kernels_<strategy>.so); other objects reused.
set -e
cd "$(dirname "$0")/.."
B=ray_community_amd/ops/_build
mkdir -p scripts/ab_lib
for S in max-ilp max-memory-clause iterative-ilp iterative-minreg; do
  mkdir -p $B/ab_$S
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c ray_community_amd/ops/csrc/attention.hip \
      -o $B/ab_$S/attention.hip.o -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=$S &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c ray_community_amd/ops/csrc/attention_dkdv.hip \
      -o $B/ab_$S/attention_dkdv.hip.o -mllvm -amdgpu-sched-strategy=$S &
done
wait
for S in max-ilp max-memory-clause iterative-ilp iterative-minreg; do
  objs=$(ls $B/*.hip.o | grep -v "/attention.hip.o\|/attention_dkdv.hip.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/ab_lib/libraca_kernels_$S.so $objs \
      $B/ab_$S/attention.hip.o $B/ab_$S/attention_dkdv.hip.o
  echo built $S
done
