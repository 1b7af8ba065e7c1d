#!/bin/bash
# Config 5 (Data map_batches GPU preprocess -> Serve bf16 replica) on 1x MI355X.
set -o pipefail
mkdir -p gpurun_out
export RCA_NO_REBUILD=1
timeout -k 10 300 python -u -c "
import time, torch
from bench_data_serve import Classifier
c = Classifier('resnet50', 224, 256, 'cuda')
x = torch.randn(256, 3, 224, 224, device='cuda', dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
for _ in range(5): c(x)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): c(x)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
print(f'replica-only resnet50 bf16 bs256 inference: {dt*1e3:.2f} ms/batch  {256/dt:.0f} img/s')
" > gpurun_out/replica_only.log 2>&1 && tail -1 gpurun_out/replica_only.log || { tail -20 gpurun_out/replica_only.log; exit 1; }
timeout -k 10 400 python -u bench_data_serve.py --batches 40 --warmup 6 > gpurun_out/bench_data_serve.log 2>&1 && tail -1 gpurun_out/bench_data_serve.log || { tail -30 gpurun_out/bench_data_serve.log; exit 1; }
