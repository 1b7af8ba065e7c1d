#!/bin/bash
# A/B: attention compiled with / without -amdgpu-mfma-vgpr-form (accumulators in AGPRs)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
ACC=$GRAFT_REPO_ROOT/ray_community_amd/ops/libraca_kernels_acc.so
RCA_KERNEL_LIB=$ACC timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -q --timeout 200 > gpurun_out/pytest_attn_acc.log 2>&1; rc=$?; echo "pytest(acc) exit $rc"; tail -2 gpurun_out/pytest_attn_acc.log
[ $rc -eq 0 ] || exit $rc
for lib in default acc; do for nh in 1 2; do
  if [ $lib = acc ]; then export RCA_KERNEL_LIB=$ACC; else unset RCA_KERNEL_LIB; fi
  RCA_ATTN_DKDV_NH=$nh timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_${lib}_nh$nh.log 2>&1 || exit 1
  echo "$lib NH=$nh: $(grep rca-hip gpurun_out/attn_${lib}_nh$nh.log)"
done; done
