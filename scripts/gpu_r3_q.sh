#!/bin/bash
# A/B of AMDGPU scheduler strategies for the attention kernels (scripts/ab_sched_build.sh)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for round in 1 2 3; do
  for S in default bias0 nopostra nocluster relaxocc; do
    if [ $S = default ]; then unset RCA_KERNEL_LIB; else export RCA_KERNEL_LIB=$GRAFT_REPO_ROOT/scripts/ab_lib/libraca_kernels_$S.so; fi
    timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/r3q_${S}_$round.log 2>&1 || { tail -5 gpurun_out/r3q_${S}_$round.log; exit 1; }
    echo "$S r$round: $(grep rca-hip gpurun_out/r3q_${S}_$round.log)"
  done
done
