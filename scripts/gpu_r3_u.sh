#!/bin/bash
# RMSNorm dw into the flat buffer + prefetched residual grad: tests, rms A/B, bench
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_ddp_norm_gpu.py -k "rmsnorm or norm or llama or adamw or embedding" > gpurun_out/r3u_tests.log 2>&1 || { tail -30 gpurun_out/r3u_tests.log; exit 1; }
tail -1 gpurun_out/r3u_tests.log
for i in 1 2 3; do
  unset RCA_KERNEL_LIB; timeout -k 10 60 python scripts/rms_bench.py 2>&1 | grep rmsnorm
  RCA_KERNEL_LIB=$GRAFT_REPO_ROOT/scripts/ab_lib/libraca_kernels_rmsold.so timeout -k 10 60 python scripts/rms_bench.py 2>&1 | grep rmsnorm
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r3u_bench.json 2> gpurun_out/r3u_bench.err || { tail -20 gpurun_out/r3u_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r3u_bench.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
