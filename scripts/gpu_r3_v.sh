#!/bin/bash
# GBDT: GPU tests (histogram kernel vs CPU reference, GPU training), kernel + training bench, rocprof stats
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/r3v_tests.log 2>&1 || { tail -40 gpurun_out/r3v_tests.log; exit 1; }
tail -3 gpurun_out/r3v_tests.log
timeout -k 10 300 python -u scripts/gbdt_bench.py > gpurun_out/r3v_bench.log 2>&1 || { tail -30 gpurun_out/r3v_bench.log; exit 1; }
cat gpurun_out/r3v_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3v_prof -o gb -- python -u scripts/gbdt_bench.py --rounds 10 > gpurun_out/r3v_prof.log 2>&1 || { tail -30 gpurun_out/r3v_prof.log; exit 1; }
f=$(find gpurun_out/r3v_prof -name "*.db" | head -1); python scripts/rocpd_summary.py "$f" 12 > gpurun_out/r3v_prof_summary.md; cat gpurun_out/r3v_prof_summary.md; find gpurun_out/r3v_prof -name "*.db" -delete
