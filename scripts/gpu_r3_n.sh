#!/bin/bash
# AdamW-fused W^T + wgrad plans: GPU tests, same-box A/B of the 8B step, per-step kernel table
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "adamw or wgrad_plans or gemm or swiglu or llama" > gpurun_out/r3n_tests.log 2>&1 || { tail -30 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
for v in new old new2; do
  if [ $v = old ]; then export RCA_ADAMW_WT=0 RCA_WGRAD_PLAN=0; else unset RCA_ADAMW_WT RCA_WGRAD_PLAN; fi
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3n_bench_$v.json 2> gpurun_out/r3n_bench_$v.err || { tail -20 gpurun_out/r3n_bench_$v.err; exit 1; }
  echo "bench $v: $(python -c "import json;d=json.loads(open('gpurun_out/r3n_bench_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['extra'])")"
done
unset RCA_ADAMW_WT RCA_WGRAD_PLAN
rm -rf gpurun_out/pd1 gpurun_out/pd4
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd1 -o run -- python scripts/prof_llama.py --steps 1 > gpurun_out/pd1.log 2>&1 || { tail gpurun_out/pd1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd4 -o run -- python scripts/prof_llama.py --steps 4 > gpurun_out/pd4.log 2>&1 || { tail gpurun_out/pd4.log; exit 1; }
grep "ms/step" gpurun_out/pd4.log
python scripts/prof_diff.py $(find gpurun_out/pd1 -name "*.db" | head -1) 1 $(find gpurun_out/pd4 -name "*.db" | head -1) 4 45 > gpurun_out/r3n_perstep.md
head -30 gpurun_out/r3n_perstep.md
rm -rf gpurun_out/pd1 gpurun_out/pd4
