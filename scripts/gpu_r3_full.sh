#!/bin/bash
# round 3 full GPU pass: every GPU test, smoke, then the headline bench (ddp) and the zero mode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3f_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r3f_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3f_smoke.log 2>&1 || { tail -20 gpurun_out/r3f_smoke.log; exit 1; }
tail -1 gpurun_out/r3f_smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3f_bench_ddp.json 2> gpurun_out/r3f_bench_ddp.err || { tail -20 gpurun_out/r3f_bench_ddp.err; exit 1; }
cat gpurun_out/r3f_bench_ddp.json
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 --parallel zero > gpurun_out/r3f_bench_zero.json 2> gpurun_out/r3f_bench_zero.err || { tail -20 gpurun_out/r3f_bench_zero.err; exit 1; }
cat gpurun_out/r3f_bench_zero.json
