#!/bin/bash
# wide (64 rows/wave) attention forward: numerics, then interleaved A/B at the 8B shape
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py \
  -k "variants or fwd_bwd or long_causal" > gpurun_out/r4o_tests.log 2>&1 && \
ATTN_WIDE_AB=1 timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/r4o_ab.log 2>&1
