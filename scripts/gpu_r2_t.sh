#!/bin/bash
# refreshed per-step kernel table (1-step vs 4-step trace difference) after the attention hazard fix + bench
# 4-step trace) of the 8B step + bench
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -2 gpurun_out/t_attn.log
rm -rf gpurun_out/pd1 gpurun_out/pd4
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd1 -o run -- python scripts/prof_llama.py --steps 1 > gpurun_out/pd1.log 2>&1 || { tail gpurun_out/pd1.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/pd4 -o run -- python scripts/prof_llama.py --steps 4 > gpurun_out/pd4.log 2>&1 || { tail gpurun_out/pd4.log; exit 1; }
grep "ms/step" gpurun_out/pd4.log
python scripts/prof_diff.py $(find gpurun_out/pd1 -name "*.db" | head -1) 1 $(find gpurun_out/pd4 -name "*.db" | head -1) 4 45 > gpurun_out/pd_summary_t.md
head -40 gpurun_out/pd_summary_t.md
rm -rf gpurun_out/pd1 gpurun_out/pd4
timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/t_bench.log 2>&1 || { tail gpurun_out/t_bench.log; exit 1; }
tail -1 gpurun_out/t_bench.log
