#!/bin/bash
# A/B the gfx950 GEMM pipeline variants (RCA_GEMM_VARIANT) on the 8B training shapes.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
for v in ${VARIANTS:-1 2 3}; do
  RCA_GEMM_VARIANT=$v timeout -k 10 300 python scripts/gemm_bench.py --rounds 2 --reps 3 ${ONLY:+--only $ONLY} \
    > gpurun_out/gemm_var$v.log 2>&1 || exit 1
  echo "variant $v"; grep -o '"name": "[a-z_]*"\|"ours_tf": [0-9.]*\|"torch+tr_tf": [0-9.]*\|"max_rel_err": [0-9.e-]*\|total_ms.*' gpurun_out/gemm_var$v.log | paste -sd' ' | sed 's/"name"/\n"name"/g'
done
