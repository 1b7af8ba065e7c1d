"""External simulators over HTTP (reference: rllib/env/policy_server_input.py, policy_client.py,
rllib/examples/envs/external_envs/cartpole_server.py / cartpole_client.py): PPO trains on CartPole
episodes that a separate client process plays through PolicyClient, with the server's policy
answering (remote inference) or the client acting on its own synced copy (local inference)."""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

import ray_community_amd as ray

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CLIENT = r'''
import sys, time
sys.path.insert(0, {root!r})
import numpy as np
from ray_community_amd.rllib.env.envs import make_vector_env
from ray_community_amd.rllib.env.policy_client import PolicyClient
client = None
for _ in range(300):
    try:
        client = PolicyClient("http://127.0.0.1:{port}", inference_mode={mode!r}, update_interval=0.5)
        break
    except Exception:
        time.sleep(0.1)
env = make_vector_env("CartPole-v1", 1, seed=7)
deadline = time.time() + {seconds}
while time.time() < deadline:
    eid = client.start_episode()
    obs, _ = env.reset()
    while True:
        a = client.get_action(eid, obs[0])
        obs, r, te, tr, info = env.step(np.asarray([a]))
        client.log_returns(eid, float(r[0]))
        if te[0] or tr[0]:
            client.end_episode(eid, info["final_obs"][0])
            break
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["remote", "local"])
def test_ppo_learns_from_external_client_process(shutdown_only, mode):
    from ray_community_amd.rllib import PPOConfig
    from ray_community_amd.rllib.env.policy_server_input import PolicyServerInput
    from ray_community_amd.rllib.utils.spaces import Box, Discrete

    port = _port()
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    hi = np.array([4.8, 10.0, 0.42, 10.0], np.float32)
    cfg = (PPOConfig().environment(None, observation_space=Box(-hi, hi, dtype=np.float32), action_space=Discrete(2))
           .offline_data(input_=lambda ioctx: PolicyServerInput(ioctx, "127.0.0.1", port))
           .env_runners(num_env_runners=0, rollout_fragment_length=1000)
           .training(lr=3e-4, train_batch_size=1000, minibatch_size=128, num_epochs=8, vf_loss_coeff=0.01,
                     model={"fcnet_hiddens": [64, 64]})
           .debugging(seed=0))
    algo = cfg.build()
    proc = subprocess.Popen([sys.executable, "-c", CLIENT.format(root=ROOT, port=port, mode=mode, seconds=240)],
                            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        first, best = None, 0.0
        t0 = time.time()
        while time.time() - t0 < 200:
            r = algo.train()
            m = r["episode_reward_mean"]
            if m == m:
                first = m if first is None else first
                best = max(best, m)
            if best > 120:
                break
        assert first is not None and best > max(2 * first, 60), (first, best)
        assert proc.poll() is None, proc.stderr.read()[-2000:]  # the client kept playing
    finally:
        proc.kill()
        algo.stop()
