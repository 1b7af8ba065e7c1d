#!/bin/bash
# Round 4: memory-instruction issue probe (stagger), hand GEMM variant 4 (staggered waves) vs 3 vs
# hipBLASLt on the 13 Llama-3-8B shapes, tightened GEMM numerics tests.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 ./scripts/probes/issue_probe 2000 > gpurun_out/issue_probe2.log 2>&1 || { tail -5 gpurun_out/issue_probe2.log; exit 1; }
cat gpurun_out/issue_probe2.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm or wgrad" > gpurun_out/r4a_tests.log 2>&1 || { tail -30 gpurun_out/r4a_tests.log; exit 1; }
tail -1 gpurun_out/r4a_tests.log
timeout -k 10 400 python -u scripts/gemm_bench.py --variants 4,3 --rounds 3 --reps 5 --json gpurun_out/r4a_gemm.json > gpurun_out/r4a_gemm.log 2>&1 || { tail -20 gpurun_out/r4a_gemm.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4a_gemm.json"))
for r in d["rows"]:
    print(f"{r['name']:11s} v4 {r['v4_tf']:7.1f}  v3 {r['v3_tf']:7.1f}  torch {r['torch_tf']:7.1f}  torch+tr {r['torch+tr_tf']:7.1f}  err4 {r['v4_err']:.1e}")
print(d["total_ms"])
PY
