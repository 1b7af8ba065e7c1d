#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_diag.py 3 > gpurun_out/r3e_diag.log 2>&1; rc=$?
cat gpurun_out/r3e_diag.log | grep -v amdgpu.ids
exit $rc
