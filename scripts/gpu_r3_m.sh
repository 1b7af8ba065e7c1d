#!/bin/bash
# GEMM layout policy measurement + fresh per-step kernel table of the current step
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/transpose_bench.py > gpurun_out/r3m_tr.log 2>&1 || { tail -20 gpurun_out/r3m_tr.log; exit 1; }
RCA_TRANSPOSE_TILE64=1 timeout -k 10 200 python -u scripts/transpose_bench.py >> gpurun_out/r3m_tr.log 2>&1 || { tail -20 gpurun_out/r3m_tr.log; exit 1; }
grep exact gpurun_out/r3m_tr.log
timeout -k 10 400 python -u scripts/gemm_policy.py > gpurun_out/r3m_policy.log 2>&1 || { tail -20 gpurun_out/r3m_policy.log; exit 1; }
cat gpurun_out/r3m_policy.log | grep name
rm -rf gpurun_out/pd1 gpurun_out/pd4
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd1 -o run -- python scripts/prof_llama.py --steps 1 > gpurun_out/pd1.log 2>&1 || { tail gpurun_out/pd1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd4 -o run -- python scripts/prof_llama.py --steps 4 > gpurun_out/pd4.log 2>&1 || { tail gpurun_out/pd4.log; exit 1; }
grep "ms/step" gpurun_out/pd4.log
python scripts/prof_diff.py $(find gpurun_out/pd1 -name "*.db" | head -1) 1 $(find gpurun_out/pd4 -name "*.db" | head -1) 4 45 > gpurun_out/r3m_perstep.md
head -30 gpurun_out/r3m_perstep.md
rm -rf gpurun_out/pd1 gpurun_out/pd4
