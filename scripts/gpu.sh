#!/bin/bash
# One parameterised launcher for GPU-box work (run under gpurun from the repo root):
#
#   scripts/gpu.sh TAG STEP [STEP ...]
#
# Every STEP runs under its own time limit, output under gpurun_out/TAG_<n>_<kind>.log, and the
# first failing step ends the call (nothing further touches the GPU after a fault or a timeout).
# STEP forms:
#   tests[:PYTEST_ARGS]        every GPU test (or the given selection), thread-method timeouts
#   smoke                      __graft_entry__.smoke()
#   bench[:BENCH_ARGS]         bench.py (default --gpus 1 --steps 20 --warmup 3); prints the JSON line
#   perstep                    1- vs 4-step rocprofv3 kernel traces of scripts/prof_llama.py, differenced
#   cpath[:PROF_ARGS]          one kernel trace; per-stream busy time + main-stream critical path (scripts/critical_path.py)
#   ab:STEP_AB_ARGS            scripts/step_ab.py: same-process interleaved A/B of the 8B step
#   py:SCRIPT ARGS             any python script
#   pmc:COUNTERS:SCRIPT ARGS   one rocprofv3 --pmc pass (kernel-trace only; counters comma-separated)
#   sh:SECONDS:COMMAND         any other command under its own limit
set -o pipefail
TAG=${1:?tag}
shift
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  log=gpurun_out/${TAG}_${n}_${kind}.log
  echo "== step $n: $step" >&2
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest ${arg:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > "$log" 2>&1
      rc=$?
      tail -3 "$log"
      [ $rc -ne 0 ] && grep -E "FAILED|Error|error" "$log" | head -20 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$log" 2>&1
      rc=$?
      tail -2 "$log" ;;
    bench)
      timeout -k 10 500 python -u bench.py ${arg:---gpus 1 --steps 20 --warmup 3} > "${log%.log}.json" 2> "$log"
      rc=$?
      [ $rc -ne 0 ] && tail -20 "$log"
      tail -1 "${log%.log}.json" | cut -c1-400 ;;
    perstep)
      rm -rf gpurun_out/pd1 gpurun_out/pd4
      timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pd1 -o run -- python scripts/prof_llama.py --steps 1 > "$log" 2>&1 &&
        timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pd4 -o run -- python scripts/prof_llama.py --steps 4 >> "$log" 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        grep "ms/step" "$log"
        python scripts/prof_diff.py "$(find gpurun_out/pd1 -name '*.db' | head -1)" 1 \
          "$(find gpurun_out/pd4 -name '*.db' | head -1)" 4 45 > "gpurun_out/${TAG}_perstep.md"
        head -26 "gpurun_out/${TAG}_perstep.md" | cut -c1-200
      else
        tail -20 "$log"
      fi
      rm -rf gpurun_out/pd1 gpurun_out/pd4 ;;
    cpath)
      # one kernel trace of warmup + 4 steps; per-stream busy time and the main-stream critical path
      rm -rf gpurun_out/cp
      timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/cp -o run -- python scripts/prof_llama.py --steps 4 --warmup 2 ${arg} > "$log" 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        grep "ms/step" "$log"
        python scripts/critical_path.py "$(find gpurun_out/cp -name '*.db' | head -1)" --steps 3 > "gpurun_out/${TAG}_cpath.md"
        head -16 "gpurun_out/${TAG}_cpath.md"
      else
        tail -20 "$log"
      fi
      rm -rf gpurun_out/cp ;;
    ab)
      timeout -k 10 1000 python -u scripts/step_ab.py $arg > "$log" 2>&1
      rc=$?
      tail -25 "$log" ;;
    py)
      timeout -k 10 600 python -u $arg > "$log" 2>&1
      rc=$?
      tail -40 "$log" ;;
    pmc)
      ctr=${arg%%:*}
      prog=${arg#*:}
      rm -rf "gpurun_out/${TAG}_pmc$n"
      timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc ${ctr//,/ } -d "gpurun_out/${TAG}_pmc$n" -o run -- python -u $prog > "$log" 2>&1
      rc=$?
      tail -5 "$log" ;;
    sh)
      secs=${arg%%:*}
      cmd=${arg#*:}
      timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
      rc=$?
      tail -30 "$log" ;;
    *)
      echo "unknown step kind: $kind" >&2
      exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $n ($step) failed: rc=$rc" >&2
    exit $rc
  fi
done
