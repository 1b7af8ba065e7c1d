"""Metrics export + dashboard JSON API (reference tests: python/ray/tests/test_metrics_agent.py,
dashboard/tests)."""
import json
import time
import urllib.request

import ray_community_amd as ray


def _get(url):
    with urllib.request.urlopen(url, timeout=10) as r:
        return r.read().decode()


def test_dashboard_metrics_and_state(shutdown_only):
    ctx = ray.init(num_cpus=2, include_dashboard=True, dashboard_port=0)
    url = ctx.dashboard_url
    assert url

    @ray.remote
    class Reporter:
        def record(self):
            from ray_community_amd.util.metrics import Counter, Gauge

            c = Counter("rca_test_requests", description="requests", tag_keys=("route",))
            c.inc(3.0, tags={"route": "/a"})
            Gauge("rca_test_queue").set(7)
            return True

    r = Reporter.remote()
    assert ray.get(r.record.remote())
    deadline = time.time() + 20
    text = ""
    while time.time() < deadline:
        text = _get(url + "/metrics")
        if "rca_test_requests" in text:
            break
        time.sleep(0.5)
    assert 'rca_test_requests{source=' in text and 'route="/a"' in text, text[-2000:]
    assert "rca_cluster_resources_total" in text and "rca_object_store_capacity_bytes" in text
    actors = json.loads(_get(url + "/api/actors"))
    assert any(a["class_name"] == "Reporter" for a in actors)
    status = json.loads(_get(url + "/api/cluster_status"))
    assert status["total"]["CPU"] == 2.0
    assert json.loads(_get(url + "/api/version"))["version"]


def test_dashboard_overview_page_logs_and_events(shutdown_only):
    ctx = ray.init(num_cpus=2, include_dashboard=True, dashboard_port=0, log_to_driver=False)
    url = ctx.dashboard_url

    @ray.remote
    def noisy():
        print("dashboard-log-line")
        return 1

    ray.get(noisy.remote())
    page = _get(url + "/")
    assert "<html" in page and "/api/actors" in page and "showLog" in page
    logs = json.loads(_get(url + "/api/logs"))
    files = [f for fs in logs.values() for f in fs]
    assert files
    deadline = time.time() + 10
    text = ""
    while time.time() < deadline and "dashboard-log-line" not in text:
        text = "".join(_get(url + f"/api/logs/file?filename={f}&lines=50") for f in files)
        time.sleep(0.1)
    assert "dashboard-log-line" in text
    ev = json.loads(_get(url + "/api/cluster_events"))
    assert any(e["source_type"] == "NODE" for e in ev)
    assert json.loads(_get(url + "/api/placement_groups")) == []


def test_state_api_over_http(shutdown_only):
    """The reference state-API HTTP protocol on the dashboard (/api/v0/<resource> with limit and
    filter_keys/predicates/values, /api/v0/<resource>/summarize, the result envelope) and the
    Python state API pointed at it with ``address=`` (what a remote ``ray list actors`` does)."""
    import requests

    from ray_community_amd.util import state

    ctx = ray.init(num_cpus=2, include_dashboard=True, dashboard_port=0)
    url = ctx.dashboard_url

    @ray.remote
    class Named:
        def ping(self):
            return 1

    a = Named.options(name="alpha").remote()
    b = Named.options(name="beta").remote()
    ray.get([a.ping.remote(), b.ping.remote()])

    @ray.remote
    def t():
        return 1

    ray.get([t.remote() for _ in range(3)])
    body = requests.get(url + "/api/v0/actors", params={"limit": 10}, timeout=10).json()
    assert body["result"] is True
    res = body["data"]["result"]
    assert res["total"] >= 2 and {r["name"] for r in res["result"]} >= {"alpha", "beta"}
    body = requests.get(url + "/api/v0/actors", params={"filter_keys": "name", "filter_predicates": "=",
                                                        "filter_values": "beta"}, timeout=10).json()
    assert [r["name"] for r in body["data"]["result"]["result"]] == ["beta"]
    assert body["data"]["result"]["num_filtered"] == 1
    lim = requests.get(url + "/api/v0/actors", params={"limit": 1}, timeout=10).json()["data"]["result"]
    assert lim["num_after_truncation"] == 1 and lim["total"] >= 2
    bad = requests.get(url + "/api/v0/actors", params={"filter_keys": "name", "filter_predicates": "~",
                                                       "filter_values": "x"}, timeout=10)
    assert bad.status_code == 400 and bad.json()["result"] is False
    summ = requests.get(url + "/api/v0/tasks/summarize", timeout=10).json()
    assert summ["result"] and "cluster" in summ["data"]["result"]["node_id_to_summary"]
    assert requests.get(url + "/api/v0/nope", timeout=10).status_code == 404
    # the Python state API against the HTTP endpoint
    names = [r["name"] for r in state.list_actors(address=url, filters=[("name", "=", "alpha")])]
    assert names == ["alpha"]
    assert len(state.list_nodes(address=url)) == 1
