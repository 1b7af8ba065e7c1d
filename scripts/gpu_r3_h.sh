#!/bin/bash
# attention backward: dQ || dK/dV stream overlap A/B (modes 0/1/2), GPU attention tests, 8B bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/r3i_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
for m in 0 1 2 1 0; do
  RCA_ATTN_BWD_OVERLAP=$m timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/r3i_attn_$m.log 2>&1 || { echo attn bench failed; tail gpurun_out/r3i_attn_$m.log; exit 1; }
  echo "mode $m: $(grep rca-hip gpurun_out/r3i_attn_$m.log)"
done
for m in 1 0; do
  RCA_ATTN_BWD_OVERLAP=$m timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3i_bench_$m.json 2> gpurun_out/r3i_bench_$m.err || { echo bench failed; tail gpurun_out/r3i_bench_$m.err; exit 1; }
  echo "bench mode $m: $(python -c "import json;d=json.loads(open('gpurun_out/r3i_bench_$m.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done
echo exit=0
