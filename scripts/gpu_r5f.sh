set -o pipefail
scripts/gpu.sh r5f "tests:tests/test_attention_gpu.py" "sh:300:ATTN_NOPS_AB=1 python -u scripts/attn_bench.py" "ab:--arms nop3,nop1 --rounds 3 --steps 10" || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5f_prof -o run -- python -u scripts/attn_bench.py > gpurun_out/r5f_prof.log 2>&1 || exit 1
find gpurun_out/r5f_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r5f_attn_kernel_stats.csv
rm -rf gpurun_out/r5f_prof
head -12 gpurun_out/r5f_attn_kernel_stats.csv | cut -c1-220
