#!/bin/bash
# GPU tests + smoke + 1-GPU bench + the ZeRO (N>1 default) path rehearsed under torchrun with an
# RCCL process group of one rank. Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 6 --warmup 2 --parallel zero > gpurun_out/bench_zero1.log 2>&1 && tail -1 gpurun_out/bench_zero1.log || { tail -30 gpurun_out/bench_zero1.log; exit 1; }
