#!/bin/bash
# A/B on one box: headline bench with the new (4 loads in flight) vs the old sumsq kernel library
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
OLD=$PWD/scripts/ab_lib/libraca_kernels_oldsumsq.so
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/x_new$r.log 2>/dev/null || exit 1
  echo "new$r $(python -c "import json;d=json.loads(open('gpurun_out/x_new$r.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  RCA_KERNEL_LIB=$OLD timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/x_old$r.log 2>/dev/null || exit 1
  echo "old$r $(python -c "import json;d=json.loads(open('gpurun_out/x_old$r.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done
