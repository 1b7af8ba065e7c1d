#!/bin/bash
# Kernel table (rocprofv3 --kernel-trace --stats, csv) of any python script:
#   scripts/gpu_kprof.sh TAG SCRIPT [ARGS...]
# -> gpurun_out/TAG_kernel_stats.csv and the top rows on stdout.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
TAG=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf "gpurun_out/${TAG}_prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof" -o run -- python -u "$@" > "gpurun_out/${TAG}_prof.log" 2>&1 || { tail -20 "gpurun_out/${TAG}_prof.log"; exit 1; }
f=$(find "gpurun_out/${TAG}_prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "gpurun_out/${TAG}_kernel_stats.csv"
t=$(find "gpurun_out/${TAG}_prof" -name "*kernel_trace.csv" | head -1)
if [ -n "$t" ] && [ -n "$TAIL_AFTER_GAP_MS" ]; then
  # steady state only: the dispatches after the last idle gap longer than TAIL_AFTER_GAP_MS (the
  # script sleeps between warm-up and its timed loop)
  python - "$t" "$TAIL_AFTER_GAP_MS" > "gpurun_out/${TAG}_tail.md" <<'PY'
import collections, csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gap = float(sys.argv[2]) * 1e6
cut, end = 0, 0
for i, r in enumerate(rows):
    s = int(r["Start_Timestamp"])
    if i and s - end > gap:
        cut = i
    end = max(end, int(r["End_Timestamp"]))
tail = rows[cut:]
agg = collections.defaultdict(lambda: [0, 0])
for r in tail:
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = sum(v[1] for v in agg.values())
span = int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])
print(f"steady-state window: {len(tail)} dispatches, kernel sum {tot / 1e6:.3f} ms, span {span / 1e6:.3f} ms\n")
print("| kernel | calls | total ms | % | avg us |\n|---|---|---|---|---|")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"| `{k[:110]}` | {n} | {t / 1e6:.3f} | {100 * t / tot:.1f} | {t / n / 1e3:.1f} |")
PY
  head -30 "gpurun_out/${TAG}_tail.md"
fi
rm -rf "gpurun_out/${TAG}_prof"
python - "gpurun_out/${TAG}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel ms {tot / 1e6:.2f}")
for r in rows[:25]:
    print(f"{r['Name'][:100]:100s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.1f} pct {float(r['Percentage']):5.1f}")
PY
