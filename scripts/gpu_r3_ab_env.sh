#!/bin/bash
# A/B: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) on the headline step, interleaved
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/ab_base_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_base_$i.json').read().strip().splitlines()[-1]);print('base', d['ms_per_step'])"
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/ab_karg_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_karg_$i.json').read().strip().splitlines()[-1]);print('devkernarg', d['ms_per_step'])"
done
