"""Per-node dashboard agents (reference: dashboard/agent.py, modules/reporter/reporter_agent.py,
modules/log/log_agent.py; tests dashboard/modules/node/tests/test_node.py and
dashboard/modules/log/tests/test_log.py): one agent process per alive node, reporting node and
worker-process stats and serving that node's logs; started / stopped with nodes and the dashboard."""
import json
import os
import time
import urllib.error
import urllib.request

import pytest

import ray_community_amd as ray


def _get(url, timeout=10):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.read().decode()


def _wait(pred, timeout=30, period=0.2):
    deadline = time.time() + timeout
    while time.time() < deadline:
        out = pred()
        if out:
            return out
        time.sleep(period)
    raise AssertionError("condition not reached")


@pytest.fixture
def dash_cluster(monkeypatch):
    monkeypatch.setenv("RCA_DASHBOARD_AGENT_PERIOD_S", "0.3")
    ctx = ray.init(num_cpus=2, include_dashboard=True, dashboard_port=0, log_to_driver=False)
    from ray_community_amd._private.worker import _state

    yield ctx, _state["head"], _state["dashboard"]
    ray.shutdown()


def _summary(url):
    return json.loads(_get(url + "/nodes?view=summary"))["data"]["summary"]


def test_agent_per_node_reports_stats_and_worker_processes(dash_cluster):
    ctx, head, dash = dash_cluster
    url = ctx.dashboard_url
    nid2 = head.add_node({"CPU": 2, "side": 1})

    @ray.remote(resources={"side": 1})
    class OnSide:
        def pid(self):
            return os.getpid()

        def node(self):
            return ray.get_runtime_context().get_node_id()

    a = OnSide.remote()
    pid = ray.get(a.pid.remote())
    assert ray.get(a.node.remote()) == nid2

    def both_report():
        s = _summary(url)
        by = {n["raylet"]["nodeId"]: n for n in s}
        ok = len(by) == 2 and all(n["agent"]["pid"] for n in by.values())
        return by if ok and any(w["pid"] == pid for w in _detail(url, nid2)["workers"]) else None

    by = _wait(both_report)
    agent_pids = {n["agent"]["pid"] for n in by.values()}
    assert len(agent_pids) == 2  # one process per node
    assert by[nid2]["raylet"]["state"] == "ALIVE" and by[nid2]["raylet"]["resources"]["side"] == 1
    assert by[nid2]["mem"][0] > 0 and by[nid2]["cpus"][0] >= 1
    det = _detail(url, nid2)
    w = [w for w in det["workers"] if w["pid"] == pid][0]
    assert w["rss"] > 0 and w["num_threads"] >= 1 and w["is_actor"]
    # the actor's process is reported by ITS node's agent only
    head_nid = [n for n, v in by.items() if v["raylet"]["isHeadNode"]][0]
    assert all(x["pid"] != pid for x in _detail(url, head_nid)["workers"])

    text = _get(url + "/metrics")
    assert f'ray_node_agent_up{{NodeId="{nid2}"}} 1' in text
    assert f'ray_component_rss_mb{{NodeId="{nid2}",' in text and f'pid="{pid}"' in text
    assert "rca_cluster_resources_total" in text  # the head's own exposition is still there
    with pytest.raises(urllib.error.HTTPError) as e:
        _get(url + "/nodes/" + "0" * 32)
    assert e.value.code == 404


def _detail(url, nid):
    return json.loads(_get(url + "/nodes/" + nid))["data"]["detail"]


def test_agent_serves_its_nodes_logs(dash_cluster):
    ctx, head, dash = dash_cluster
    url = ctx.dashboard_url
    nid2 = head.add_node({"CPU": 1, "side": 1})

    @ray.remote(resources={"side": 1})
    def shout():
        print("hello-from-side-node", flush=True)
        return os.getpid()

    pid = ray.get(shout.remote())

    def side_logs():
        try:
            out = json.loads(_get(f"{url}/api/v0/logs?node_id={nid2}"))
        except urllib.error.HTTPError:
            return None
        names = out["data"]["result"][nid2]
        return names or None

    names = _wait(side_logs)
    texts = {}
    for n in names:
        texts[n] = _get(f"{url}/api/v0/logs/file?node_id={nid2}&filename={n}&lines=50")
    assert any("hello-from-side-node" in t for t in texts.values()), (pid, names)
    # a file of another node is refused by this node's agent
    head_nid = [n["NodeID"] for n in ray.nodes() if n["IsHead"]][0]
    head_names = json.loads(_get(f"{url}/api/v0/logs?node_id={head_nid}"))["data"]["result"][head_nid]
    foreign = [n for n in head_names if n not in names]
    if foreign:
        with pytest.raises(urllib.error.HTTPError) as e:
            _get(f"{url}/api/v0/logs/file?node_id={nid2}&filename={foreign[0]}")
        assert e.value.code == 404


def test_agents_follow_node_membership_and_restart(dash_cluster):
    import psutil

    ctx, head, dash = dash_cluster
    sup = dash.agents
    nid2 = head.add_node({"CPU": 1})
    _wait(lambda: nid2 in sup.procs and len(sup.procs) == 2)
    p2 = sup.procs[nid2]
    _wait(lambda: nid2 in sup.reports())
    # an agent that dies is restarted
    p2.kill()
    p2.wait(10)
    _wait(lambda: sup.procs.get(nid2) is not None and sup.procs[nid2].pid != p2.pid)
    assert sup.restarts >= 1
    # a removed node's agent is stopped
    p2b = sup.procs[nid2]
    head.remove_node(nid2)
    _wait(lambda: nid2 not in sup.procs and p2b.poll() is not None)
    _wait(lambda: nid2 not in sup.reports())  # its report is withdrawn with it
    # shutdown stops every agent
    procs = list(sup.procs.values())
    assert procs
    ray.shutdown()
    for p in procs:
        assert p.poll() is not None
        assert not psutil.pid_exists(p.pid) or psutil.Process(p.pid).status() == psutil.STATUS_ZOMBIE
