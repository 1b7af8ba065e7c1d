#!/bin/bash
# Round 4 closing GPU pass on the final tree (compiled-DAG result buffering, native worker pool): every GPU test, smoke and the headline bench.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4u_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4u_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4u_smoke.log 2>&1 || { tail -20 gpurun_out/r4u_smoke.log; exit 1; }
tail -1 gpurun_out/r4u_smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r4u_bench.json 2> gpurun_out/r4u_bench.err || { tail -20 gpurun_out/r4u_bench.err; exit 1; }
tail -1 gpurun_out/r4u_bench.json | cut -c1-300
