#!/bin/bash
# flash-attention numerics + microbenchmark (dK/dV variants A/B via RCA_ATTN_DKDV_NH)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py tests/test_ops_gpu.py -q --timeout 200 > gpurun_out/pytest_attn.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
for nh in 1 2; do
  RCA_ATTN_DKDV_NH=$nh timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench_nh$nh.log 2>&1 || exit 1
  echo "NH=$nh: $(grep rca-hip gpurun_out/attn_bench_nh$nh.log)"
done
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
