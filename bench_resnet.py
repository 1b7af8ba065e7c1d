#!/usr/bin/env python3
"""Secondary benchmark: Ray Train TorchTrainer ResNet-50 DDP bf16 (BASELINE.json config
"Ray Train TorchTrainer ResNet-50 DDP bf16 on 1xMI355X"), images/s for the whole job.

    python bench_resnet.py --gpus N --steps K --warmup W [--batch-size B]

Same launch contract as bench.py (N>1 under torch.distributed.run, one rank per GPU over RCCL).
Synthetic uint8 224x224 images normalised on the GPU inside the step; random-init weights.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256, help="per GPU")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))

    import ray_community_amd as ray
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.torch import TorchTrainer
    from ray_community_amd.train.vision import resnet_train_loop_per_worker

    if world <= 1:
        ray.init(include_dashboard=False, log_to_driver=False)  # stdout: one JSON line
    cfg = {"batch_size": a.batch_size, "image_size": a.image_size, "steps": a.steps, "warmup": a.warmup,
           "device": a.device}
    trainer = TorchTrainer(resnet_train_loop_per_worker, train_loop_config=cfg,
                           scaling_config=ScalingConfig(num_workers=max(1, world), use_gpu=a.device == "cuda"),
                           run_config=RunConfig(name="bench_resnet", storage_path="/tmp/rca_bench"))
    m = trainer.fit().metrics
    if rank == 0:
        print(json.dumps({
            "metric": "ray_train_images_per_sec_resnet50_ddp", "value": round(m["images_per_s"], 1), "unit": "images/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(m["ms_per_step"], 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random uint8 images, random-init weights)",
            "config": {"model": "resnet50", "global_batch": a.batch_size * world, "image_size": a.image_size,
                       "parallelism": f"dp{world}", "optimizer": "SGD momentum 0.9 (flat)"},
            "extra": {"loss": round(m["loss"], 4), "peak_mem_gb": round(m["mem_gb"], 2)}}), flush=True)
    if world > 1:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
    if ray.is_initialized():
        ray.shutdown()


if __name__ == "__main__":
    main()
