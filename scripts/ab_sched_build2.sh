#!/bin/bash
# Second-round attention build A/B on top of iterative-ILP scheduling: scheduler metric bias,
# no post-RA scheduler, no memop clustering (scripts/ab_lib/libraca_kernels_<name>.so).
set -e
cd "$(dirname "$0")/.."
B=ray_community_amd/ops/_build
mkdir -p scripts/ab_lib
rm -f scripts/ab_lib/*.so
declare -A V
V[bias0]="-mllvm -amdgpu-schedule-metric-bias=0"
V[nopostra]="-mllvm -enable-post-misched=0"
V[nocluster]="-mllvm -misched-cluster=0"
V[relaxocc]="-mllvm -amdgpu-schedule-relaxed-occupancy"
for S in "${!V[@]}"; do
  mkdir -p $B/ab_$S
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c ray_community_amd/ops/csrc/attention.hip \
      -o $B/ab_$S/attention.hip.o -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=iterative-ilp ${V[$S]} &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c ray_community_amd/ops/csrc/attention_dkdv.hip \
      -o $B/ab_$S/attention_dkdv.hip.o -mllvm -amdgpu-sched-strategy=iterative-ilp ${V[$S]} &
done
wait
objs=$(ls $B/*.hip.o | grep -v "/attention.hip.o\|/attention_dkdv.hip.o")
for S in "${!V[@]}"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/ab_lib/libraca_kernels_$S.so $objs \
      $B/ab_$S/attention.hip.o $B/ab_$S/attention_dkdv.hip.o
  echo built $S
done
