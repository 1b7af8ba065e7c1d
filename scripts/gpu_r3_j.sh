#!/bin/bash
# delta fused into dQ: attention GPU tests, attention bench, 8B bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/r3j_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r3j_tests.log; exit 1; }
tail -2 gpurun_out/r3j_tests.log
for i in 1 2; do timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/r3j_attn_$i.log 2>&1 || { echo attn bench failed; tail gpurun_out/r3j_attn_$i.log; exit 1; }; grep rca-hip gpurun_out/r3j_attn_$i.log; done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || { echo bench failed; tail gpurun_out/r3j_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r3j_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['extra'])"
echo exit=0
