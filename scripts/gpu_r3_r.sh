#!/bin/bash
# iterative-ILP attention build + wide-grid RMSNorm dw reduction: numerics tests, bench, per-step table
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_ops_gpu.py -k "attention or attn or rmsnorm or llama" > gpurun_out/r3r_tests.log 2>&1 || { tail -30 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/r3r_attn.log 2>&1 || exit 1; grep rca-hip gpurun_out/r3r_attn.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r3r_bench.json 2> gpurun_out/r3r_bench.err || { tail -20 gpurun_out/r3r_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r3r_bench.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
rm -rf gpurun_out/pd1 gpurun_out/pd4
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd1 -o run -- python scripts/prof_llama.py --steps 1 > gpurun_out/pd1.log 2>&1 || { tail gpurun_out/pd1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd4 -o run -- python scripts/prof_llama.py --steps 4 > gpurun_out/pd4.log 2>&1 || { tail gpurun_out/pd4.log; exit 1; }
grep "ms/step" gpurun_out/pd4.log
python scripts/prof_diff.py $(find gpurun_out/pd1 -name "*.db" | head -1) 1 $(find gpurun_out/pd4 -name "*.db" | head -1) 4 45 > gpurun_out/r3r_perstep.md
head -28 gpurun_out/r3r_perstep.md
rm -rf gpurun_out/pd1 gpurun_out/pd4
