#!/bin/bash
# segmented AdamW (grid-stride) vs flat on the 8B layout, GPU tests, same-box step A/B
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "adamw or wgrad_plans" > gpurun_out/r3o_tests.log 2>&1 || { tail -30 gpurun_out/r3o_tests.log; exit 1; }
tail -1 gpurun_out/r3o_tests.log
timeout -k 10 300 python -u scripts/adamw_seg_bench.py > gpurun_out/r3o_adamw.log 2>&1 || { tail -20 gpurun_out/r3o_adamw.log; exit 1; }
tail -1 gpurun_out/r3o_adamw.log
for v in new old; do
  if [ $v = old ]; then export RCA_ADAMW_WT=0; else unset RCA_ADAMW_WT; fi
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3o_bench_$v.json 2> gpurun_out/r3o_bench_$v.err || { tail -20 gpurun_out/r3o_bench_$v.err; exit 1; }
  echo "bench $v: $(python -c "import json;d=json.loads(open('gpurun_out/r3o_bench_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done
