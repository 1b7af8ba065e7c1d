"""Reference-export parity pieces: workflow sleep / wait_for_event, StateApiClient, DAG plot,
multiprocessing TimeoutError, air ResourceRequest, RLlib TorchPolicy / ExternalEnv / aliases."""
import threading
import time

import numpy as np
import pytest

import ray_community_amd as ray


def test_workflow_sleep_and_event(shutdown_only, tmp_path):
    from ray_community_amd import workflow

    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    workflow.init(str(tmp_path / "wf"))

    @ray.remote
    def after(x, y=None):
        return ("done", x)

    t0 = time.time()
    out = workflow.run(after.bind(workflow.sleep(0.5)), workflow_id="sleepy")
    assert out[0] == "done" and time.time() - t0 >= 0.45
    assert workflow.get_status("sleepy") == workflow.WorkflowStatus.SUCCESSFUL

    class Ready(workflow.EventListener):
        async def poll_for_event(self, payload):
            return {"payload": payload}

    got = workflow.run(after.bind(workflow.wait_for_event(Ready, "evt-1")), workflow_id="evt")
    assert got == ("done", {"payload": "evt-1"})
    with pytest.raises(TypeError):
        workflow.wait_for_event(object)


def test_state_api_client_and_dag_plot(shutdown_only, tmp_path):
    from ray_community_amd.dag import InputNode, plot
    from ray_community_amd.util.state import StateApiClient

    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)

    @ray.remote
    class A:
        def f(self, x):
            return x + 1

    a = A.remote()
    ray.get(a.f.remote(1))
    c = StateApiClient()
    rows = c.list("actors")
    assert rows and c.get("actors", rows[0]["actor_id"])["class_name"] == "A"
    assert "cluster" in c.summary("tasks")

    @ray.remote
    def g(x):
        return x * 2

    with InputNode() as inp:
        dag = g.bind(g.bind(inp))
    path = plot(dag, str(tmp_path / "d.dot"))
    text = open(path).read()
    assert text.startswith("digraph") and text.count("->") == 2


def test_multiprocessing_timeout_error(shutdown_only):
    from ray_community_amd.util.multiprocessing import Pool, TimeoutError

    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    with Pool(processes=1) as p:
        r = p.apply_async(time.sleep, (2,))
        with pytest.raises(TimeoutError):
            r.get(timeout=0.2)


def test_air_resource_request():
    from ray_community_amd.air import AcquiredResources, ResourceRequest

    rr = ResourceRequest([{"CPU": 1}, {"GPU": 1}])
    assert rr.required_resources == {"CPU": 1, "GPU": 1} and not rr.head_bundle_is_empty
    assert AcquiredResources(rr).annotate_remote_entities([1, 2]) == [1, 2]


def test_torch_policy_and_external_env():
    from ray_community_amd.rllib import ExternalEnv, IMPALA, RolloutWorker, TorchPolicy
    from ray_community_amd.rllib.algorithms import Impala
    from ray_community_amd.rllib.env.envs import CartPoleVec

    assert Impala is IMPALA and RolloutWorker is not None
    env = CartPoleVec(num_envs=2)
    pol = TorchPolicy(env.observation_space, env.action_space, {})
    obs = np.zeros((3, 4), dtype=np.float32)
    acts, _, info = pol.compute_actions(obs)
    assert acts.shape == (3,) and info["vf_preds"].shape == (3,)
    a, _, _ = pol.compute_single_action(obs[0], explore=False)
    w = pol.get_weights()
    pol.set_weights(w)

    class Serving(ExternalEnv):
        def run(self):
            eid = self.start_episode()
            total = 0
            for t in range(3):
                act = self.get_action(eid, np.full(4, t, dtype=np.float32))
                total += int(act)
                self.log_returns(eid, 1.0)
            self.end_episode(eid, np.zeros(4, dtype=np.float32))
            self.result = total

    ext = Serving(env.action_space, env.observation_space)
    base = ext.to_base_env()
    steps = 0
    while True:
        obs, rew, term, trunc, infos, off = base.poll(timeout=10)
        assert obs, "external env stalled"
        done = [e for e, d in term.items() if d]
        if done:
            assert rew[done[0]] == 1.0  # the last step's return arrives with the episode end
            break
        base.send_actions({eid: 1 for eid in obs})
        steps += 1
    ext.join(5)
    assert steps == 3 and ext.result == 3
