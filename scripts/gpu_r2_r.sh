#!/bin/bash
# GEMM: default hipBLASLt heuristic vs the round-1 TunableOp table, then a fresh tuning pass over all
# training layouts (incl. the transposed-operand ones)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONPATH=$PWD
timeout -k 10 300 python -u scripts/gemm_tune.py --table ray_community_amd/ops/tuned/gemm_mi355x.csv > gpurun_out/r_table.log 2>&1; rc=$?; tail -27 gpurun_out/r_table.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/gemm_tuned2.csv
timeout -k 10 700 python -u scripts/gemm_tune.py --tune --out gpurun_out/gemm_tuned2.csv > gpurun_out/r_tune.log 2>&1; rc=$?; tail -27 gpurun_out/r_tune.log; exit $rc
