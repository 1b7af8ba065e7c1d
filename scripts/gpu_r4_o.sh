#!/bin/bash
# 64-row attention forward variants (wide, hand-scheduled): numerics first (own time limit), then
# the default kernel's tests, then an interleaved A/B at the 8B shape
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 150 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_attention_gpu.py \
  -k "variants or large_logits" > gpurun_out/r4o_tests.log 2>&1 && \
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py \
  >> gpurun_out/r4o_tests.log 2>&1 && \
ATTN_WIDE_AB=1 timeout -k 10 200 python -u scripts/attn_bench.py > gpurun_out/r4o_ab.log 2>&1
