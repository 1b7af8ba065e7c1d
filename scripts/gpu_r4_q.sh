#!/bin/bash
# Round 4 full GPU pass (4, after the core ref-pinning and Data fusion fixes): every GPU test, smoke, the headline bench
# and the per-step kernel table.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4q_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4q_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4q_smoke.log 2>&1 || { tail -20 gpurun_out/r4q_smoke.log; exit 1; }
tail -1 gpurun_out/r4q_smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r4q_bench.json 2> gpurun_out/r4q_bench.err || { tail -20 gpurun_out/r4q_bench.err; exit 1; }
tail -1 gpurun_out/r4q_bench.json | cut -c1-200
rm -rf gpurun_out/pd1 gpurun_out/pd4
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pd1 -o run -- python scripts/prof_llama.py --steps 1 > gpurun_out/pd1.log 2>&1 || { tail gpurun_out/pd1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pd4 -o run -- python scripts/prof_llama.py --steps 4 > gpurun_out/pd4.log 2>&1 || { tail gpurun_out/pd4.log; exit 1; }
grep "ms/step" gpurun_out/pd4.log
python scripts/prof_diff.py $(find gpurun_out/pd1 -name "*.db" | head -1) 1 $(find gpurun_out/pd4 -name "*.db" | head -1) 4 45 > gpurun_out/r4q_perstep.md
head -24 gpurun_out/r4q_perstep.md | cut -c1-200
rm -rf gpurun_out/pd1 gpurun_out/pd4
