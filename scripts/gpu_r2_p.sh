#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONPATH=$PWD
timeout -k 10 200 python -u scripts/diag/fwd_det.py > gpurun_out/p_fwd.log 2>&1; rc=$?; tail -20 gpurun_out/p_fwd.log; exit $rc
