#!/bin/bash
# Fused down-dgrad + SwiGLU-backward GEMM: numerics, schedule A/B, and the 8B step with/without it.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_swiglu_tr_gpu.py tests/test_ops_gpu.py -k "swiglu or gemm" > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -1 gpurun_out/r4l_tests.log
timeout -k 10 400 python -u scripts/gemm_bench.py --variants 78,79,80 --tn --rounds 3 --reps 5 --json gpurun_out/r4l_gemm.json > gpurun_out/r4l_gemm.log 2>&1 || { tail -20 gpurun_out/r4l_gemm.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4l_gemm.json"))
for r in d["rows"]:
    print(f"{r['name']:11s} " + " ".join(f"{v} {r[v + '_tn_tf']:7.1f}" for v in ["v78", "v79", "v80", "torch"]))
print({k: v for k, v in d["total_ms"].items() if k.endswith("_tn")})
print("max err", max(v for r in d["rows"] for k, v in r.items() if k.endswith("_err")))
PY
