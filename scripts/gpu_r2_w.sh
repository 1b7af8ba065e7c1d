#!/bin/bash
# compiled-DAG GPU tensor edges (TorchTensorType over HIP-IPC device slots)
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dag_device.py tests/test_dag.py > gpurun_out/w_dag.log 2>&1; rc=$?; tail -12 gpurun_out/w_dag.log; exit $rc
