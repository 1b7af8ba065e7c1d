"""Declarative Serve: config schema, ``serve build|deploy|status|config|shutdown`` CLI and the
``/api/serve/applications/`` REST API (reference: serve/tests/test_schema.py, test_cli.py,
dashboard/modules/serve/tests/test_serve_dashboard.py)."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest
import requests
import yaml
from pydantic import ValidationError

from ray_community_amd.serve.schema import ServeDeploySchema, parse_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

APP_SRC = textwrap.dedent('''
    from ray_community_amd import serve


    @serve.deployment
    class Doubler:
        def __init__(self):
            self.k = 2

        def reconfigure(self, cfg):
            self.k = int(cfg.get("k", 2))

        def __call__(self, x):
            return self.k * x


    @serve.deployment
    class Ingress:
        def __init__(self, d):
            self.d = d

        async def __call__(self, request):
            x = int(request.query_params["x"])
            return {"y": await self.d.remote(x)}


    app = Ingress.bind(Doubler.bind())


    def builder(args):
        return Ingress.bind(Doubler.options(num_replicas=int(args.get("n", 1))).bind())
''')


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_schema_validation():
    ok = parse_config({"applications": [{"name": "a", "import_path": "m:app", "route_prefix": "/a",
                                         "deployments": [{"name": "D", "num_replicas": 2}]}]})
    assert ok.applications[0].deployments[0].num_replicas == 2
    single = parse_config({"import_path": "m.app"})  # a one-application file
    assert single.applications[0].name == "default"
    bad = [
        {"applications": [{"import_path": "noseparator"}]},
        {"applications": [{"import_path": "m:a", "route_prefix": "x"}]},
        {"applications": [{"import_path": "m:a", "deployments": [{"name": "D", "num_replicas": 2,
                                                                     "autoscaling_config": {"max_replicas": 3}}]}]},
        {"applications": [{"name": "a", "import_path": "m:a"}, {"name": "a", "import_path": "m:b",
                                                                 "route_prefix": "/b"}]},
        {"applications": [{"import_path": "m:a", "deployments": [{"name": "D"}, {"name": "D"}]}]},
        {"applications": [{"import_path": "m:a", "bogus_field": 1}]},
    ]
    for b in bad:
        with pytest.raises(ValidationError):
            ServeDeploySchema.model_validate(b)


def test_serve_build_writes_a_deployable_config(tmp_path):
    (tmp_path / "myapp_b.py").write_text(APP_SRC)
    out = tmp_path / "cfg.yaml"
    r = subprocess.run([sys.executable, "-m", "ray_community_amd", "serve", "build", "myapp_b:app", "--app-dir",
                        str(tmp_path), "-o", str(out)], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    cfg = parse_config(str(out))
    deps = {d.name: d for d in cfg.applications[0].deployments}
    assert set(deps) == {"Ingress", "Doubler"} and deps["Doubler"].num_replicas == 1
    assert cfg.applications[0].import_path == "myapp_b:app"


def _cli(args, env, timeout=180):
    return subprocess.run([sys.executable, "-m", "ray_community_amd"] + args, cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_cli_deploy_status_rest_update_delete(tmp_path):
    """Deploy a two-deployment app from YAML through the CLI, query it over HTTP, read status
    from the CLI and the REST API, re-PUT it with more replicas and a new user_config (no
    restart of the untouched ingress), then DELETE it."""
    appdir = tmp_path / "code"
    appdir.mkdir()
    (appdir / "myapp_e2e.py").write_text(APP_SRC)
    http_port, dash_port = _free_port(), _free_port()
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    env.pop("RAY_ADDRESS", None)
    env["RCA_TEMP_DIR"] = str(tmp_path / "rt")
    head = subprocess.Popen([sys.executable, "-m", "ray_community_amd", "start", "--head", "--block", "--num-cpus",
                             "4", "--temp-dir", str(tmp_path / "rt"), "--include-dashboard", "--dashboard-port",
                             str(dash_port)], cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.STDOUT)
    dash = f"http://127.0.0.1:{dash_port}"
    try:
        deadline = time.time() + 120
        while True:
            try:
                if requests.get(dash + "/api/version", timeout=2).ok:
                    break
            except requests.RequestException:
                pass
            assert head.poll() is None and time.time() < deadline, "head did not come up"
            time.sleep(0.3)
        assert requests.get(dash + "/api/serve/applications/", timeout=10).json()["applications"] == {}
        cfg = {"http_options": {"host": "127.0.0.1", "port": http_port},
               "applications": [{"name": "app1", "route_prefix": "/app1", "import_path": "myapp_e2e:app",
                                 "runtime_env": {"working_dir": str(appdir)},
                                 "deployments": [{"name": "Doubler", "num_replicas": 2}]}]}
        path = tmp_path / "serve.yaml"
        path.write_text(yaml.safe_dump(cfg))
        r = _cli(["serve", "deploy", str(path)], env)
        assert r.returncode == 0, r.stderr + r.stdout

        deadline = time.time() + 120
        while True:
            st = yaml.safe_load(_cli(["serve", "status"], env).stdout)
            app = st["applications"].get("app1") or {}
            if app.get("status") == "RUNNING":
                break
            assert time.time() < deadline, st
            time.sleep(0.5)
        assert app["deployments"]["Doubler"]["target_num_replicas"] == 2
        assert requests.get(f"http://127.0.0.1:{http_port}/app1", params={"x": 21}, timeout=30).json() == {"y": 42}

        conf = yaml.safe_load(_cli(["serve", "config"], env).stdout)
        assert conf["import_path"] == "myapp_e2e:app" and conf["deployments"][0]["num_replicas"] == 2

        det = requests.get(dash + "/api/serve/applications/", timeout=10).json()
        d = det["applications"]["app1"]
        assert d["status"] == "RUNNING" and d["deployed_app_config"]["import_path"] == "myapp_e2e:app"
        assert len(d["deployments"]["Doubler"]["replicas"]) == 2
        ingress_replicas = [x["replica_id"] for x in d["deployments"]["Ingress"]["replicas"]]

        cfg["applications"][0]["deployments"] = [{"name": "Doubler", "num_replicas": 3, "user_config": {"k": 3}}]
        r = requests.put(dash + "/api/serve/applications/", json=cfg, timeout=180)
        assert r.status_code == 200, r.text
        deadline = time.time() + 120
        while True:
            d = requests.get(dash + "/api/serve/applications/", timeout=10).json()["applications"]["app1"]
            if len(d["deployments"]["Doubler"]["replicas"]) == 3 and d["status"] == "RUNNING":
                break
            assert time.time() < deadline, d
            time.sleep(0.5)
        assert d["deployments"]["Doubler"]["target_num_replicas"] == 3
        assert [x["replica_id"] for x in d["deployments"]["Ingress"]["replicas"]] == ingress_replicas
        deadline = time.time() + 60
        while requests.get(f"http://127.0.0.1:{http_port}/app1", params={"x": 5}, timeout=30).json() != {"y": 15}:
            assert time.time() < deadline
            time.sleep(0.3)

        bad = requests.put(dash + "/api/serve/applications/", json={"applications": [{"import_path": "nosep"}]},
                           timeout=30)
        assert bad.status_code == 400

        assert requests.delete(dash + "/api/serve/applications/", timeout=120).status_code == 200
        assert requests.get(dash + "/api/serve/applications/", timeout=10).json()["applications"] == {}
    finally:
        head.terminate()
        try:
            head.wait(timeout=30)
        except subprocess.TimeoutExpired:
            head.kill()
