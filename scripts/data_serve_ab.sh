#!/bin/bash
# Same-box interleaved A/B of bench_data_serve.py: the round-3 tree (_ab/r3, exported with
# `git archive 7ab7978` and built in-tree) against the current tree, ROUNDS rounds each.
#   scripts/data_serve_ab.sh TAG [ROUNDS] [EXTRA BENCH ARGS...]
set -o pipefail
TAG=${1:?tag}
ROUNDS=${2:-3}
shift 2
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
ROOT=$(pwd)
for r in $(seq 1 "$ROUNDS"); do
  for arm in r3 cur; do
    dir=$ROOT
    [ "$arm" = r3 ] && dir=$ROOT/_ab/r3
    log=$ROOT/gpurun_out/${TAG}_${arm}_${r}.log
    (cd "$dir" && timeout -k 10 300 python -u bench_data_serve.py "$@" > "$log" 2>&1)
    rc=$?
    echo "$arm round $r rc=$rc $(grep -o '"value": [0-9.]*' "$log" | head -1)"
    [ $rc -ne 0 ] && { tail -20 "$log"; exit $rc; }
  done
done
exit 0
