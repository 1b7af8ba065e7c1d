#!/bin/bash
# attention staging-store remap: numerics + microbench + PMC conflicts
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/attn_bench_k.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/a -o run --output-format csv -- python scripts/pmc_kernels.py > gpurun_out/pmc_a.log 2>&1 || exit 1
mkdir -p gpurun_out/pmc/b gpurun_out/pmc/c
python scripts/pmc_summary.py gpurun_out/pmc 2>/dev/null | grep -i "attn\|kernel |" | head -8
