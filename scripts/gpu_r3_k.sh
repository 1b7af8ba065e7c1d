#!/bin/bash
# same-box A/B: fused delta-in-dQ (current library) vs separate delta kernel (scripts/ab_lib)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "spill or pinned or owner_death" > gpurun_out/r3k_tests.log 2>&1 || { tail -30 gpurun_out/r3k_tests.log; exit 1; }
tail -2 gpurun_out/r3k_tests.log
OLD=$GRAFT_REPO_ROOT/scripts/ab_lib/libraca_kernels_delta_kernel.so
for i in 1 2; do
  timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/r3k_new_$i.log 2>&1 || exit 1; echo "fused  : $(grep rca-hip gpurun_out/r3k_new_$i.log)"
  RCA_KERNEL_LIB=$OLD timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/r3k_old_$i.log 2>&1 || exit 1; echo "separate: $(grep rca-hip gpurun_out/r3k_old_$i.log)"
done
for v in new old; do
  if [ $v = old ]; then export RCA_KERNEL_LIB=$OLD; else unset RCA_KERNEL_LIB; fi
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3k_bench_$v.json 2> gpurun_out/r3k_bench_$v.err || { tail gpurun_out/r3k_bench_$v.err; exit 1; }
  echo "bench $v: $(python -c "import json;d=json.loads(open('gpurun_out/r3k_bench_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done
echo exit=0
