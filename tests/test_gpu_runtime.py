"""Runtime features on a real MI355X: GPU actors, HBM-resident GPU objects (HIP IPC hand-off),
TorchTrainer on a GPU worker, RCCL collective group."""
import os

import pytest
import torch

import ray_community_amd as ray

pytestmark = pytest.mark.gpu


@pytest.fixture
def ray_gpu():
    ray.init(num_cpus=4, num_gpus=1)
    yield
    ray.shutdown()


def test_gpu_actor_sees_one_device(ray_gpu):
    @ray.remote(num_gpus=1)
    class G:
        def info(self):
            import torch

            return ray.get_gpu_ids(), torch.cuda.device_count(), os.environ.get("HIP_VISIBLE_DEVICES")

    ids, n, vis = ray.get(G.remote().info.remote())
    assert ids == [0] and n == 1 and vis


def test_gpu_object_ipc_handoff(ray_gpu):
    @ray.remote(num_gpus=1)
    class Producer:
        def make(self, n):
            import torch

            self.t = torch.arange(n, device="cuda", dtype=torch.float32)
            return self.t * 2  # stays in HBM; exported by HIP IPC handle

    p = Producer.remote()
    ref = p.make.remote(1 << 20)
    t = ray.get(ref)  # driver maps the producer's HBM allocation
    assert t.is_cuda
    assert float(t[-1].item()) == 2 * ((1 << 20) - 1)
    local = torch.ones(4, device="cuda")
    r2 = ray.put(local)
    assert torch.equal(ray.get(r2), local)


def test_torch_trainer_gpu_worker(ray_gpu, tmp_path):
    from ray_community_amd.train import RunConfig, ScalingConfig
    from ray_community_amd.train.llm import llama_train_loop_per_worker
    from ray_community_amd.train.torch import TorchTrainer

    t = TorchTrainer(llama_train_loop_per_worker,
                     train_loop_config={"model": "llama3-tiny", "seq_len": 128, "micro_batch": 2, "steps": 3,
                                        "warmup": 1},
                     scaling_config=ScalingConfig(num_workers=1, use_gpu=True),
                     run_config=RunConfig(name="gpu_tiny", storage_path=str(tmp_path)))
    r = t.fit()
    assert r.metrics["tokens_per_s"] > 0 and r.metrics["world_size"] == 1


def test_rccl_collective_group_single_rank(ray_gpu):
    @ray.remote(num_gpus=1)
    class W:
        def go(self):
            import torch

            from ray_community_amd.util import collective as col

            col.init_collective_group(1, 0, backend="nccl", group_name="g1")
            t = torch.ones(8, device="cuda")
            col.allreduce(t, group_name="g1")
            col.barrier(group_name="g1")
            return t.sum().item()

    assert ray.get(W.remote().go.remote()) == 8.0


def test_ppo_gpu_learner_synthetic_atari(ray_gpu):
    from ray_community_amd.rllib import PPOConfig

    cfg = (PPOConfig().environment("ALE/Pong-v5").env_runners(num_env_runners=1, num_envs_per_env_runner=4)
           .training(train_batch_size=256, minibatch_size=128, num_epochs=1).resources(num_gpus=1))
    algo = cfg.build()
    assert algo.learner_group.local.device.type == "cuda"
    r = algo.train()
    assert r["num_env_steps_sampled_this_iter"] == 256
    algo.stop()


def test_ppo_lstm_gpu_learner(ray_gpu):
    """Recurrent PPO with the learner on the GPU: chunked sequence replay + LSTM backward on HIP."""
    from ray_community_amd.rllib import PPOConfig

    cfg = (PPOConfig().environment("StatelessCartPole-v1").env_runners(num_envs_per_env_runner=8)
           .training(train_batch_size=512, minibatch_size=128, num_epochs=2,
                     model={"use_lstm": True, "lstm_cell_size": 32, "max_seq_len": 16, "fcnet_hiddens": [32]})
           .resources(num_gpus=1))
    algo = cfg.build()
    try:
        assert algo.learner_group.local.device.type == "cuda"
        for _ in range(2):
            r = algo.train()
        info = r["info"]["learner"]["default_policy"]
        assert r["num_env_steps_sampled_this_iter"] == 512 and info["num_minibatches"] > 0
        assert all(v == v for v in (info["total_loss"], info["vf_loss"]))  # finite, not NaN
    finally:
        algo.stop()


def test_gpu_object_store_spill_and_restore_bit_exact():
    """HBM budget 48 MB: putting 4 x 16 MB GPU objects pushes the least recently used ones to
    pinned host memory (hipMemcpyAsync on a side stream); get() restores them into HBM bit-exact."""
    ray.init(num_cpus=2, num_gpus=1, _system_config={"gpu_object_store_memory": 48 << 20})
    try:
        from ray_community_amd._private import worker as w

        head = w._state["head"]
        g = torch.Generator(device="cuda").manual_seed(0)
        vals = [torch.randn(4 << 20, device="cuda", generator=g) for _ in range(4)]  # 16 MB each
        keep = [v.cpu() for v in vals]
        refs = [ray.put(v) for v in vals]
        del vals
        import time

        deadline = time.time() + 30
        while time.time() < deadline and head.rpc_gpu_store_stats("t")["num_spilled"] < 1:
            time.sleep(0.05)
        st = head.rpc_gpu_store_stats("t")
        assert st["num_spilled"] >= 1 and st["usage"].get("0", 0) <= 48 << 20
        for r, k in zip(refs, keep):
            out = ray.get(r)
            assert out.is_cuda and torch.equal(out.cpu(), k)
        assert head.rpc_gpu_store_stats("t")["num_restored"] >= 1
    finally:
        ray.shutdown()


def test_gpu_store_pinned_pool_and_concurrent_spill_restore():
    """Spill / restore run outside the store lock on pooled pinned buffers: a second spill cycle
    reuses the pool (no new hipHostMalloc), objects spill and restore concurrently from threads,
    and every restore is bit-exact (incl. a channels-last tensor's strides)."""
    import threading

    from ray_community_amd._private.gpu_store import GpuObjectStore
    from ray_community_amd._private.serialization import serialize

    st = GpuObjectStore()
    g = torch.Generator(device="cuda").manual_seed(0)
    vals = [torch.randn(1 << 20, device="cuda", generator=g) for _ in range(6)]
    vals.append(torch.randn(4, 8, 5, 7, device="cuda", generator=g).contiguous(memory_format=torch.channels_last))
    keep = [v.cpu() for v in vals]
    oids = [bytes([i]) * 20 for i in range(len(vals))]
    for o, v in zip(oids, vals):
        st.add(o, serialize(v), copy=True)
    for cycle in range(2):
        errs = []

        def worker(idx):
            try:
                for i in idx:
                    assert st.spill(oids[i]) > 0
                for i in idx:
                    assert st.restore(oids[i]) is not None
            except Exception as e:  # noqa
                errs.append(e)

        th = [threading.Thread(target=worker, args=(list(range(k, len(oids), 3)),)) for k in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert not errs, errs
        for o, k in zip(oids, keep):
            t = st.local_tensor({"oid": o, "slot": 0})
            assert t is not None and torch.equal(t.cpu(), k) and t.stride() == k.stride()
    s = st.stats()
    assert s["num_spilled"] == 2 * len(oids) and s["num_restored"] == 2 * len(oids)
    assert s["pinned_pool_hits"] >= len(oids)  # cycle 2 took every buffer from the pool
    st.free(oids)


def test_gpu_object_owner_death_is_object_lost(ray_gpu):
    """A GPU object lives in its owner's HBM: once the owner dies, readers get ObjectLostError."""
    from ray_community_amd import exceptions as exc

    @ray.remote(num_gpus=1)
    class Producer:
        def make(self):
            import torch

            return torch.full((1024,), 3.0, device="cuda")

        def pid(self):
            return os.getpid()

    p = Producer.remote()
    r1 = p.make.remote()
    assert float(ray.get(r1).sum().item()) == 3.0 * 1024  # zero-copy IPC map of the owner's HBM
    r2 = p.make.remote()
    ray.wait([r2])
    ray.kill(p)
    import time

    time.sleep(1.0)
    with pytest.raises(exc.ObjectLostError):
        ray.get(r2, timeout=30)


@pytest.mark.gpu
def test_gpu_object_keeps_channels_last_layout():
    """A channels-last activation handed to another GPU actor arrives channels-last (same
    strides, same values): NCHW bytes would silently switch the consumer's conv kernels."""
    import torch

    import ray_community_amd as ray

    ray.init(num_cpus=4, num_gpus=1)
    try:
        @ray.remote(num_gpus=0.25)
        class Reader:
            def check(self, x):
                return (x.is_contiguous(memory_format=torch.channels_last), tuple(x.stride()),
                        x.float().sum().item())

        x = torch.randn(4, 3, 16, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = Reader.remote()
        cl, stride, s = ray.get(r.check.remote(x))
        assert cl and stride == tuple(x.stride())
        assert abs(s - x.float().sum().item()) < 1e-2
        ref = ray.put(x)
        assert ray.get(r.check.remote(ref))[1] == tuple(x.stride())
    finally:
        ray.shutdown()


def test_max_calls_task_returns_cuda_tensor(ray_gpu):
    """A ``max_calls=1`` GPU task's worker retires after the call, but the CUDA tensor it
    returned lives in that worker's GPU object store: the process must stay until the reader is
    done with it (exiting at once would turn the result into OwnerDiedError)."""
    @ray.remote(num_gpus=1, max_calls=1)
    def make(n):
        import torch

        return torch.full((n,), 3.0, device="cuda")

    refs = [make.remote(1 << 16) for _ in range(2)]
    import time

    time.sleep(1.0)  # the retiring workers have long sent their completions
    for r in refs:
        t = ray.get(r)
        assert t.is_cuda and float(t.sum().item()) == 3.0 * (1 << 16)
    del t, refs


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (peer import over xGMI)")
def test_gpu_object_peer_import_between_gpus():
    """Actor on GPU a produces a CUDA tensor; an actor on GPU b maps it through the GPU object
    store's HIP IPC import (peer access over xGMI) and reads it bit-exactly."""
    ray.init(num_cpus=4, num_gpus=2)
    try:
        @ray.remote(num_gpus=1)
        class P:
            def make(self, n):
                import torch

                return torch.arange(n, device="cuda", dtype=torch.float32) * 3

            def dev(self):
                return ray.get_gpu_ids()

        @ray.remote(num_gpus=1)
        class C:
            def check(self, t, n):
                import torch

                return t.is_cuda, float(t[-1].item()), bool(torch.equal(t.cpu(), torch.arange(n).float() * 3))

            def dev(self):
                return ray.get_gpu_ids()

        p, c = P.remote(), C.remote()
        assert ray.get(p.dev.remote()) != ray.get(c.dev.remote())
        n = 1 << 20
        is_cuda, last, same = ray.get(c.check.remote(p.make.remote(n), n))
        assert is_cuda and last == 3.0 * (n - 1) and same
    finally:
        ray.shutdown()


def _rccl_rank(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    res = {}
    for dt in (torch.bfloat16, torch.float32):
        g = torch.Generator(device="cuda").manual_seed(1234)
        full = [torch.randn(4096, 129, device="cuda", generator=g).to(dt) for _ in range(world)]  # every rank's input
        mine = full[rank].clone()
        dist.all_reduce(mine)
        ref = torch.stack([f.float() for f in full]).sum(0)
        tol = 2e-2 if dt == torch.bfloat16 else 1e-5
        res[f"allreduce_{dt}"] = bool(torch.allclose(mine.float(), ref, atol=tol, rtol=tol))
        rs = torch.empty(4096 // world, 129, device="cuda", dtype=dt)
        dist.reduce_scatter_tensor(rs, full[rank].clone())
        res[f"reduce_scatter_{dt}"] = bool(torch.allclose(rs.float(), ref.chunk(world)[rank], atol=tol, rtol=tol))
        ag = torch.empty(world * 4096, 129, device="cuda", dtype=dt)
        dist.all_gather_into_tensor(ag, full[rank])
        res[f"all_gather_{dt}"] = bool(torch.equal(ag, torch.cat(full)))
    torch.cuda.synchronize()
    if rank == 0:
        import json

        with open(os.path.join(out_dir, "rccl.json"), "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL over xGMI)")
def test_rccl_two_ranks_collectives_match_torch(tmp_path):
    """Two processes, one GPU each, RCCL: all-reduce / reduce-scatter / all-gather of bf16 and
    fp32 tensors against sums computed on one device."""
    import json
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_rccl_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = json.load(open(os.path.join(tmp_path, "rccl.json")))
    assert res and all(res.values()), res


def test_dqn_frame_stacking_connector_gpu_learner(ray_gpu):
    """Atari-style DQN: single 84x84 frames from the env, stacked to 4 by the FrameStacking
    env-to-module connector on the off-policy path; the CNN Q-learner trains on the GPU."""
    import numpy as np

    from ray_community_amd.rllib import DQNConfig
    from ray_community_amd.rllib.connectors.env_to_module import FrameStackingEnvToModule

    cfg = (DQNConfig().environment("ALE/Pong-v5", env_config={"frame_stack": 1})
           .env_runners(num_env_runners=1, num_envs_per_env_runner=4,
                        env_to_module_connector=lambda env: [FrameStackingEnvToModule(num_frames=4)])
           .training(train_batch_size=32, num_steps_sampled_before_learning_starts=64, target_network_update_freq=100)
           .resources(num_gpus=1))
    algo = cfg.build()
    try:
        assert algo.obs_space.shape == (84, 84, 4)
        assert algo.learner_group.local.device.type == "cuda"
        for _ in range(6):
            r = algo.train()
        assert r["timesteps_total"] >= 64 and np.isfinite(r["info"]["learner"]["default_policy"]["loss"])
    finally:
        algo.stop()
