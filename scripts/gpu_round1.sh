#!/bin/bash
# first GPU check: kernel numerics, a quick 1B bench, then the 8B headline bench
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?"
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --model llama3-1b --steps 5 --warmup 2 > gpurun_out/bench_1b.log 2>&1 || { echo "bench 1b failed"; tail -30 gpurun_out/bench_1b.log; exit 1; }
tail -3 gpurun_out/bench_1b.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_8b.log 2>&1 || { echo "bench 8b failed"; tail -30 gpurun_out/bench_8b.log; exit 1; }
tail -3 gpurun_out/bench_8b.log
