#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1 PYTHONPATH=$PWD
timeout -k 10 200 python -u scripts/diag/norm_det.py > gpurun_out/o_norm.log 2>&1; rc=$?; cat gpurun_out/o_norm.log | tail -30; [ $rc -eq 0 ] || exit $rc
AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u scripts/diag/norm_det.py > gpurun_out/o_norm_ser.log 2>&1; rc=$?; echo SERIALIZED; tail -12 gpurun_out/o_norm_ser.log; exit $rc
