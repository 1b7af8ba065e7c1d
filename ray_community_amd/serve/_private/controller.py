"""Serve controller (reference: ``serve/_private/{controller,deployment_state,application_state,
autoscaling_policy}.py``). A detached async actor owning every application's deployments:
reconciles replica actors to the target count, health-checks them, applies user_config updates,
and runs the autoscaling loop on the ongoing-request metric."""
from __future__ import annotations

import asyncio
import math
import time
from typing import Any, Dict, List, Optional

CONTROLLER_NAME = "SERVE_CONTROLLER_ACTOR"
NAMESPACE = "serve"


class _DeploymentState:
    def __init__(self, app, name, spec):
        self.app = app
        self.name = name
        self.spec = spec
        self.replicas: Dict[str, Any] = {}  # tag -> actor handle
        self.members = 0  # bumped on every change of ``replicas`` (routers long-poll it)
        self.version = 0
        self.target = spec["num_replicas"]
        self.status = "UPDATING"
        self.message = ""
        self.last_scale = 0.0
        self.counter = 0
        self.unhealthy_since = {}
        self.health: Dict[str, float] = {}  # tag -> time of the last passed health check
        self.pgs: Dict[str, Any] = {}  # tag -> the replica's placement group (placement_group_bundles)
        self.nodes: Dict[str, str] = {}  # tag -> node id it was pinned to (max_replicas_per_node)
        # tag -> {"node_id", "gpus"}: where the replica runs (node and physical GPU ids), reported by
        # the replica once it is up; routers prefer same-node / same-GPU replicas with it
        self.locations: Dict[str, Dict] = {}


class ServeController:
    def __init__(self, http_options: Optional[Dict] = None):
        self.apps: Dict[str, Dict[str, _DeploymentState]] = {}
        self.app_meta: Dict[str, Dict] = {}
        self.http_options = http_options or {}
        self._loop_task = None
        self.proxy = None
        self.handle_queues: Dict[tuple, Dict[str, tuple]] = {}  # (app, dep) -> router id -> (n, ts)
        self._draining: Dict[str, asyncio.Future] = {}  # tag -> background drain-and-kill of a stopped replica

    async def _ensure_loop(self):
        if self._loop_task is None:
            self._loop_task = asyncio.ensure_future(self._control_loop())

    # ------------------------------------------------------------------ deploy
    async def deploy_application(self, app_name: str, deployments: List[Dict], ingress: str, route_prefix: Optional[str],
                                 app_config: Optional[Dict] = None):
        """Create or update one application. ``app_config``: the declarative config it came from
        (``ServeApplicationSchema`` dict; ``serve config`` / the REST API report it back)."""
        await self._ensure_loop()
        for meta_app, meta in self.app_meta.items():
            if meta_app != app_name and route_prefix is not None and meta.get("route_prefix") == route_prefix:
                raise ValueError(f"route_prefix {route_prefix!r} is already used by application {meta_app!r}")
        old = self.apps.get(app_name, {})
        new = {}
        for spec in deployments:
            st = old.get(spec["name"])
            if st is None:
                st = _DeploymentState(app_name, spec["name"], spec)
            else:
                if st.spec.get("code_version") and spec.get("code_version"):  # both from a config
                    code_changed = st.spec["code_version"] != spec["code_version"]
                else:
                    code_changed = st.spec["body_hash"] != spec["body_hash"] or \
                        st.spec["init_args_blob"] != spec["init_args_blob"]
                code_changed = code_changed or st.spec["actor_options"] != spec["actor_options"]
                if code_changed:  # old replicas drain in the background while new ones start
                    await self._stop_replicas(st, list(st.replicas))
                elif spec.get("user_config") != st.spec.get("user_config"):
                    from ..._private.worker import _core

                    await asyncio.gather(*[r.reconfigure.remote(spec.get("user_config")) for r in st.replicas.values()])
                st.spec = spec
                st.status = "UPDATING"
            st.target = spec["num_replicas"] if not spec.get("autoscaling_config") else max(
                spec["autoscaling_config"].get("initial_replicas") or spec["autoscaling_config"].get("min_replicas", 1),
                1 if not st.replicas else len(st.replicas))
            new[spec["name"]] = st
        for name, st in old.items():
            if name not in new:
                await self._stop_replicas(st, list(st.replicas))
        self.apps[app_name] = new
        self.app_meta[app_name] = {"ingress": ingress, "route_prefix": route_prefix, "status": "DEPLOYING",
                                   "deployed_at": time.time(), "config": app_config}
        await self._reconcile_all()
        return True

    async def wait_app_running(self, app_name: str, timeout_s: float = 120.0):
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            await self._reconcile_all()
            meta = self.app_meta.get(app_name)
            if meta is None:
                return "NOT_STARTED"
            if meta["status"] in ("RUNNING", "DEPLOY_FAILED"):
                return meta["status"]
            await asyncio.sleep(0.05)
        return self.app_meta.get(app_name, {}).get("status", "NOT_STARTED")

    async def delete_application(self, app_name: str):
        deps = self.apps.pop(app_name, {})
        self.app_meta.pop(app_name, None)
        # this call (not the control loop) waits for the replicas to drain
        await asyncio.gather(*[self._stop_replicas(st, list(st.replicas), wait=True) for st in deps.values()])
        return True

    async def shutdown(self):
        for app in list(self.apps):
            await self.delete_application(app)
        if self._loop_task is not None:
            self._loop_task.cancel()
        return True

    # ------------------------------------------------------------------ replicas
    async def _start_replica(self, st: _DeploymentState):
        from ...actor import ActorClass
        from .replica import ServeReplica

        spec = st.spec
        opts = dict(spec["actor_options"])
        mc = spec.get("max_ongoing_requests", 5)
        opts["max_concurrency"] = max(mc, 1) + 4
        opts.setdefault("num_cpus", 0)
        node = None
        if spec.get("max_replicas_per_node"):
            node = self._pick_node(st)
            if node is None:
                st.message = (f"replicas pending: no node can take another replica under "
                              f"max_replicas_per_node={spec['max_replicas_per_node']}")
                return None
        st.counter += 1
        tag = f"{st.app}#{st.name}#{st.counter}"
        pg = None
        if spec.get("placement_group_bundles"):
            # reference deployment_scheduler.py: one placement group per replica, actor in bundle 0,
            # the replica's child tasks/actors captured into the other bundles
            from ...util.placement_group import placement_group
            from ...util.scheduling_strategies import PlacementGroupSchedulingStrategy

            pg = placement_group(spec["placement_group_bundles"], strategy=spec.get("placement_group_strategy") or "PACK")
            opts["scheduling_strategy"] = PlacementGroupSchedulingStrategy(
                pg, placement_group_bundle_index=0, placement_group_capture_child_tasks=True)
            st.pgs[tag] = pg
        elif node is not None:
            from ...util.scheduling_strategies import NodeAffinitySchedulingStrategy

            opts["scheduling_strategy"] = NodeAffinitySchedulingStrategy(node, soft=False)
            st.nodes[tag] = node
        cls = ActorClass(ServeReplica, opts)
        r = cls.remote(st.app, st.name, tag, spec["body"], spec["init_args"], spec["init_kwargs"],
                       spec.get("user_config"), spec["is_function"], logging_config=spec.get("logging_config"),
                       max_ongoing_requests=mc)
        st.replicas[tag] = r
        self._bump(st)
        asyncio.ensure_future(self._fetch_location(st, tag, r))
        return tag, r

    async def _fetch_location(self, st: _DeploymentState, tag: str, r):
        try:
            loc = await r.location.remote()
        except Exception:  # the replica died before answering: nothing to record
            return
        if tag in st.replicas:
            st.locations[tag] = loc
            self._bump(st)

    def _pick_node(self, st: _DeploymentState) -> Optional[str]:
        """A node for one more replica under ``max_replicas_per_node``: alive, big enough for the
        replica's resources, below the cap; the one holding the fewest replicas (spread)."""
        from ..._private.worker import nodes

        cap = int(st.spec["max_replicas_per_node"])
        opts = st.spec.get("actor_options") or {}
        need = {"CPU": float(opts.get("num_cpus", 0) or 0), "GPU": float(opts.get("num_gpus", 0) or 0)}
        need.update({k: float(v) for k, v in (opts.get("resources") or {}).items()})
        counts: Dict[str, int] = {}
        for t in st.replicas:
            n = st.nodes.get(t)
            if n is not None:
                counts[n] = counts.get(n, 0) + 1
        best = None
        for n in nodes():
            if not n.get("Alive", True):
                continue
            nid = n["NodeID"]
            c = counts.get(nid, 0)
            res = n.get("Resources") or {}
            if c >= cap or any(v > 0 and res.get(k, 0.0) < v for k, v in need.items()):
                continue
            if best is None or (c, nid) < best[0]:
                best = ((c, nid), nid)
        return None if best is None else best[1]

    def _bump(self, st):
        """The replica set of ``st`` changed: wake every router long-polling it."""
        st.members += 1
        ev = getattr(self, "_members_ev", None)
        if ev is not None:
            ev.set()
        self._members_ev = asyncio.Event()

    async def listen_replicas(self, app_name: str, deployment: str, known: int, timeout_s: float = 10.0):
        """Long poll (reference: serve/_private/long_poll.py LongPollHost): returns the replica set
        as soon as its membership counter differs from ``known``, or ``{"unchanged": True}`` after
        ``timeout_s``; None once the deployment is gone."""
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout_s
        while True:
            st = self.apps.get(app_name, {}).get(deployment)
            if st is None:
                return None
            if st.members != known:
                info = await self.get_replicas(app_name, deployment)
                info["members"] = st.members
                return info
            rem = deadline - loop.time()
            if rem <= 0:
                return {"unchanged": True, "members": known}
            if getattr(self, "_members_ev", None) is None:
                self._members_ev = asyncio.Event()
            try:
                await asyncio.wait_for(self._members_ev.wait(), rem)
            except asyncio.TimeoutError:
                pass

    async def _stop_replicas(self, st, tags, wait: bool = False):
        """Take replicas out of routing NOW; each drains and is killed by a background task
        (reference deployment_state.py: STOPPING replicas are polled by the state machine, so one
        slow drain never stalls reconciliation of other deployments). ``wait``: also await them."""
        tasks = [self._stop_replica(st, t) for t in tags]
        tasks = [x for x in tasks if x is not None]
        if wait and tasks:
            await asyncio.gather(*tasks, return_exceptions=True)

    def _stop_replica(self, st, t):
        r = st.replicas.pop(t, None)
        if r is None:
            return None
        self._bump(st)
        st.health.pop(t, None)
        st.nodes.pop(t, None)
        pg = st.pgs.pop(t, None)
        loop_s = float(st.spec.get("graceful_shutdown_wait_loop_s", 2.0))
        timeout_s = float(st.spec.get("graceful_shutdown_timeout_s", 20.0))
        task = asyncio.ensure_future(self._drain_and_kill(r, pg, loop_s, timeout_s))
        self._draining[t] = task
        task.add_done_callback(lambda _f, t=t: self._draining.pop(t, None))
        return task

    async def _drain_and_kill(self, r, pg, loop_s: float, timeout_s: float):
        # graceful shutdown (reference replica.py perform_graceful_shutdown): the replica is
        # already out of the routing table; it drains its ongoing requests, polling every
        # graceful_shutdown_wait_loop_s, and is killed after graceful_shutdown_timeout_s
        try:
            await asyncio.wait_for(r.prepare_for_shutdown.remote(loop_s, timeout_s), timeout_s + 5)
        except Exception:
            pass
        self._kill_replica(r, pg)

    @staticmethod
    def _kill_replica(r, pg):
        from ..._private.worker import kill

        try:
            kill(r)
        except Exception:
            pass
        if pg is not None:
            from ...util.placement_group import remove_placement_group

            try:
                remove_placement_group(pg)
            except Exception:
                pass

    async def num_draining(self):
        return len(self._draining)

    async def get_replica_placement(self, app_name: str, deployment: str):
        """{replica tag: {"node_id", "placement_group_id"}} (placement tests / the dashboard)."""
        st = self.apps.get(app_name, {}).get(deployment)
        if st is None:
            return None
        return {t: {"node_id": st.nodes.get(t),
                    "placement_group_id": st.pgs[t].id.hex() if t in st.pgs else None} for t in st.replicas}

    async def _reconcile_all(self):
        for app, deps in list(self.apps.items()):
            healthy_all = True
            failed = False
            for st in deps.values():
                cur = len(st.replicas)
                if cur < st.target:
                    for _ in range(st.target - cur):
                        if await self._start_replica(st) is None:
                            break  # no node can take it now (max_replicas_per_node): retried next round
                elif cur > st.target:
                    await self._stop_replicas(st, list(st.replicas)[st.target:])
                # readiness + periodic health checks: a replica is checked until it first passes
                # (constructor still running: a timeout is "not ready yet"), then every
                # health_check_period_s; after that a failed or timed-out check (> health_check_
                # timeout_s) replaces it (reference deployment_state.py check_health)
                period = float(st.spec.get("health_check_period_s", 10.0))
                hto = float(st.spec.get("health_check_timeout_s", 30.0))
                now = time.time()
                due = [(tag, r) for tag, r in list(st.replicas.items())
                       if tag not in st.health or now - st.health[tag] >= period]
                results = await asyncio.gather(*[asyncio.wait_for(r.check_health.remote(), hto) for _, r in due],
                                               return_exceptions=True)
                for (tag, r), res in zip(due, results):
                    if not isinstance(res, BaseException):
                        st.health[tag] = time.time()
                        continue
                    if isinstance(res, asyncio.TimeoutError) and tag not in st.health:
                        continue  # never ready yet
                    st.message = f"replica {tag} failed its health check: {type(res).__name__}: {res}"
                    if st.replicas.pop(tag, None) is not None:
                        self._bump(st)
                    st.health.pop(tag, None)
                    st.nodes.pop(tag, None)
                    failed = True
                    self._kill_replica(r, st.pgs.pop(tag, None))
                ready = sum(1 for tag in st.replicas if tag in st.health)
                if ready >= st.target and st.target > 0:
                    st.status = "HEALTHY"
                elif failed:
                    st.status = "UNHEALTHY"
                    healthy_all = False
                else:
                    healthy_all = False
            meta = self.app_meta.get(app)
            if meta is not None:
                if healthy_all:
                    meta["status"] = "RUNNING"
                elif failed and meta["status"] == "DEPLOYING":
                    meta["status"] = "DEPLOY_FAILED"

    async def _control_loop(self):
        while True:
            try:
                await self._autoscale()
                await self._reconcile_all()
            except Exception:
                pass
            await asyncio.sleep(0.5)

    async def _autoscale(self):
        now = time.time()
        for deps in self.apps.values():
            for st in deps.values():
                ac = st.spec.get("autoscaling_config")
                if not ac or not st.replicas:
                    continue
                try:
                    counts = await asyncio.gather(*[r.get_num_ongoing.remote() for r in st.replicas.values()])
                except Exception:
                    continue
                now_q = time.time()
                queued = sum(n for n, ts in self.handle_queues.get((st.app, st.name), {}).values()
                             if now_q - ts < 30.0)
                total = sum(counts) + queued
                target_per = ac.get("target_ongoing_requests", ac.get("target_num_ongoing_requests_per_replica", 2))
                desired = math.ceil(total / max(target_per, 1e-9)) if total > 0 else ac.get("min_replicas", 1)
                desired = max(ac.get("min_replicas", 1), min(ac.get("max_replicas", 1), desired))
                cur = st.target
                if desired > cur and now - st.last_scale >= ac.get("upscale_delay_s", 0.0):
                    st.target = desired
                    st.last_scale = now
                elif desired < cur and now - st.last_scale >= ac.get("downscale_delay_s", 5.0):
                    st.target = desired
                    st.last_scale = now

    async def record_handle_queue(self, app_name: str, deployment: str, router_id: str, n: int):
        self.handle_queues.setdefault((app_name, deployment), {})[router_id] = (n, time.time())
        return True

    # ------------------------------------------------------------------ queries
    async def get_replicas(self, app_name: str, deployment: str):
        st = self.apps.get(app_name, {}).get(deployment)
        if st is None:
            return None
        return {"replicas": list(st.replicas.items()), "max_ongoing_requests": st.spec.get("max_ongoing_requests", 5),
                "locations": {t: st.locations[t] for t in st.replicas if t in st.locations},
                "max_queued_requests": st.spec.get("max_queued_requests", -1), "version": st.version,
                "members": st.members}

    async def get_ingress(self, app_name: str):
        meta = self.app_meta.get(app_name)
        return None if meta is None else meta["ingress"]

    async def list_applications(self):
        """{application name: ingress deployment} of every deployed application (gRPC routing)."""
        return {app: m["ingress"] for app, m in self.app_meta.items()}

    async def list_routes(self):
        return {m["route_prefix"]: (app, m["ingress"]) for app, m in self.app_meta.items() if m["route_prefix"]}

    async def status(self):
        out = {}
        for app, deps in self.apps.items():
            meta = self.app_meta.get(app, {})
            out[app] = {"status": meta.get("status"), "route_prefix": meta.get("route_prefix"),
                        "deployments": {n: {"status": st.status, "replicas": len(st.replicas),
                                            "target": st.target, "message": st.message}
                                        for n, st in deps.items()}}
        return out

    async def set_deploy_config(self, config: Dict):
        self.deploy_config = config
        return True

    async def get_app_configs(self):
        """{app: the declarative config it was deployed from} (apps deployed from code: None)."""
        return {app: m.get("config") for app, m in self.app_meta.items()}

    async def get_serve_instance_details(self):
        """The ``GET /api/serve/applications/`` body (reference ``ServeInstanceDetails``):
        instance options, and per application its status, route, deployed config and, per
        deployment, status, target and live replicas."""
        apps = {}
        for app, deps in self.apps.items():
            meta = self.app_meta.get(app, {})
            dd = {}
            for n, st in deps.items():
                cfg = {k: st.spec.get(k) for k in ("num_replicas", "max_ongoing_requests", "user_config",
                                                    "autoscaling_config")}
                cfg["name"] = n
                cfg["ray_actor_options"] = st.spec.get("actor_options") or {}
                dd[n] = {"name": n, "status": st.status, "message": st.message, "target_num_replicas": st.target,
                         "deployment_config": cfg,
                         "replicas": [{"replica_id": tag, "state": "RUNNING"} for tag in st.replicas]}
            apps[app] = {"name": app, "route_prefix": meta.get("route_prefix"), "status": meta.get("status"),
                         "message": "", "last_deployed_time_s": meta.get("deployed_at"),
                         "deployed_app_config": meta.get("config"), "docs_path": None, "deployments": dd}
        dc = getattr(self, "deploy_config", None) or {}
        return {"controller_info": {"actor_name": CONTROLLER_NAME}, "proxy_location": dc.get("proxy_location",
                                                                                             "EveryNode"),
                "http_options": dc.get("http_options") or self.http_options or None,
                "grpc_options": dc.get("grpc_options"),
                "proxies": {"head": {"status": "HEALTHY", **(self.proxy or {})}} if self.proxy else {},
                "deploy_mode": "MULTI_APP", "applications": apps, "target_capacity": dc.get("target_capacity")}

    async def set_proxy(self, info):
        self.proxy = info
        return True

    async def get_proxy(self):
        return self.proxy
