#!/bin/bash
# Variant-7 schedule A/B (71-73) on the TN layout + PMC passes of variant 7 vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u scripts/gemm_bench.py --variants 76,77,78 --tn --rounds 3 --reps 5 --json gpurun_out/r4g_gemm.json > gpurun_out/r4g_gemm.log 2>&1 || { tail -20 gpurun_out/r4g_gemm.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4g_gemm.json"))
for r in d["rows"]:
    print(f"{r['name']:11s} " + " ".join(f"{v} {r[v + '_tn_tf']:7.1f}" for v in ["v76", "v77", "v78", "torch"]))
print({k: v for k, v in d["total_ms"].items() if k.endswith("_tn")})
print("max err", max(v for r in d["rows"] for k, v in r.items() if k.endswith("_err")))
PY

