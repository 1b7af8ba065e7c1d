#!/bin/bash
# Attention microbenchmark kernel table (rocprofv3 --kernel-trace --stats, csv) at the 8B shape.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
TAG=${1:-attn}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf "gpurun_out/${TAG}_prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof" -o run -- python -u scripts/attn_bench.py > "gpurun_out/${TAG}_prof.log" 2>&1 || { tail -20 "gpurun_out/${TAG}_prof.log"; exit 1; }
f=$(find "gpurun_out/${TAG}_prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "gpurun_out/${TAG}_kernel_stats.csv"
rm -rf "gpurun_out/${TAG}_prof"
python - "gpurun_out/${TAG}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
