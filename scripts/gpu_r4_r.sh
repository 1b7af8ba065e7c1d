#!/bin/bash
# headline step A/B: default attention forward vs the hand-scheduled 64-row one (RCA_ATTN_FWD=hs),
# interleaved, 20 timed steps each
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
for r in 1 2; do
  for m in default hs; do
    if [ $m = hs ]; then export RCA_ATTN_FWD=hs; else unset RCA_ATTN_FWD; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r4r_${m}_$r.json 2> gpurun_out/r4r_${m}_$r.err || exit 1
    echo "$m $r $(tail -1 gpurun_out/r4r_${m}_$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
