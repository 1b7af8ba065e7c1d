#!/bin/bash
# Hand-scheduled dK/dV (RCA_ATTN_DKDV=hs): equivalence with the compiler-scheduled kernel, the
# attention numerics with it, then A/B timing.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py -k hand_scheduled > gpurun_out/r4m_eq.log 2>&1; tail -15 gpurun_out/r4m_eq.log | grep -E "passed|failed|assert|Error" | head -12
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log | grep -E "assert|Error|FAILED" | head; exit 1; }
tail -1 gpurun_out/r4m_tests.log
for i in 1 2; do
RCA_ATTN_DKDV=hs timeout -k 10 120 python -u scripts/attn_bench.py 2>&1 | grep rca-hip | sed 's/^/hs   /'
timeout -k 10 120 python -u scripts/attn_bench.py 2>&1 | grep rca-hip | sed 's/^/base /'
done
