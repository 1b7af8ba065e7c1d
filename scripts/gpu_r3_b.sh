#!/bin/bash
# GEMM A/B: gemm4 (2) vs gemm4 without in-loop LDS-DMA (91, timing diagnostic only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/gemm_bench.py --rounds 3 --reps 5 --variants 2,91 --json gpurun_out/r3b_gemm.json > gpurun_out/r3b_gemm.log 2>&1
rc=$?
cat gpurun_out/r3b_gemm.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{\"name'):
        r=json.loads(l); print(r['name'], r['v2_tf'], r['v91_tf'], r['torch+tr_tf'])
    elif 'total' in l: print(l.strip())
"
exit $rc
