"""External simulators over HTTP, server side (reference: ``rllib/env/policy_server_input.py:28``).

``PolicyServerInput`` is an input reader: an HTTP server on the env runner that external
simulators talk to through ``PolicyClient`` (``policy_client.py``). The runner's training loop
reads SampleBatches from it instead of stepping an env:

    config.environment(observation_space=..., action_space=...)
          .offline_data(input_=lambda ioctx: PolicyServerInput(ioctx, "127.0.0.1", 9900))
          .env_runners(num_env_runners=0)

Commands (one JSON POST each): ``START_EPISODE``, ``GET_ACTION`` (remote inference: the server's
current policy answers), ``LOG_ACTION`` (the client acted itself, e.g. local inference, sending
the policy outputs it used), ``LOG_RETURNS``, ``END_EPISODE``, ``GET_WORKER_ARGS`` (spaces and
model config for a client-side policy copy) and ``GET_WEIGHTS``.

A serving thread polls the episodes (an ``ExternalEnv`` underneath), answers pending
observations in one batched forward pass of the runner's module, and turns every finished
episode into transitions (obs, action, action_logp, vf_preds, reward, ...). ``next()`` hands out
the finished episodes, concatenated into one env-major ``[1, T]`` fragment with the episode ends
marked terminal, once at least ``rollout_fragment_length`` steps are in.
"""
from __future__ import annotations

import collections
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, Optional

import numpy as np
import torch

from ..policy.sample_batch import SampleBatch
from .external_env import ExternalEnv

START_EPISODE = "START_EPISODE"
GET_ACTION = "GET_ACTION"
LOG_ACTION = "LOG_ACTION"
LOG_RETURNS = "LOG_RETURNS"
END_EPISODE = "END_EPISODE"
GET_WORKER_ARGS = "GET_WORKER_ARGS"
GET_WEIGHTS = "GET_WEIGHTS"


def _jsonable(x):
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().tolist()
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    return x


class IOContext:
    """What an input reader factory gets (reference ``rllib/offline/io_context.py``): the config
    and the env runner (``worker``) whose module answers the actions."""

    def __init__(self, config: Dict, worker=None, worker_index: int = 0):
        self.config = config
        self.worker = worker
        self.worker_index = worker_index


class _ServerEnv(ExternalEnv):
    def run(self):  # clients drive the episodes through the HTTP handler
        while True:
            time.sleep(3600)


class PolicyServerInput(ThreadingHTTPServer):
    daemon_threads = True

    def __init__(self, ioctx: IOContext, address: str, port: int, idle_timeout: float = 3.0):
        self.ioctx = ioctx
        self.worker = ioctx.worker
        cfg = ioctx.config or {}
        self.fragment_length = int(cfg.get("rollout_fragment_length", 200) or 200)
        self.env = _ServerEnv(self.worker.action_space, self.worker.observation_space,
                              max_concurrent=int(cfg.get("max_concurrent_episodes", 1000)))
        self.base_env = self.env.to_base_env()
        self.idle_timeout = idle_timeout
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        self._open: Dict[str, Dict] = {}  # episode id -> {"rows": [...], "pending": (obs, act, logp, vf, logits)}
        self._ready: "collections.deque" = collections.deque()  # finished episodes' transition rows
        self._ready_steps = 0
        self._returns: "collections.deque" = collections.deque()
        self.episodes_finished = 0
        super().__init__((address, int(port)), self._handler_class())
        self._serve_t = threading.Thread(target=self.serve_forever, name="policy-server-http", daemon=True)
        self._serve_t.start()
        self._loop_t = threading.Thread(target=self._serving_loop, name="policy-server-loop", daemon=True)
        self._loop_t.start()

    # ------------------------------------------------------------------ HTTP
    def _handler_class(self):
        server = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                try:
                    req = json.loads(self.rfile.read(n).decode())
                    resp = server._execute(req)
                    body, code = json.dumps(_jsonable(resp)).encode(), 200
                except Exception as e:  # noqa
                    body, code = json.dumps({"error": f"{type(e).__name__}: {e}"}).encode(), 500
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        return Handler

    def _execute(self, req: Dict):
        cmd = req["command"]
        env = self.env
        if cmd == START_EPISODE:
            eid = env.start_episode(req.get("episode_id"), req.get("training_enabled", True))
            with self._cv:
                self._open[eid] = {"rows": [], "pending": None, "reward": 0.0, "train": req.get("training_enabled", True)}
            return {"episode_id": eid}
        if cmd == GET_ACTION:
            return {"action": env.get_action(req["episode_id"], np.asarray(req["observation"], np.float32))}
        if cmd == LOG_ACTION:
            # the client acted (local inference / its own controller): its policy outputs ride along
            eid = req["episode_id"]
            obs = np.asarray(req["observation"], np.float32)
            extra = req.get("extra") or {}
            with self._cv:
                self._close_pending(eid)
                ep = self._open[eid]
                if "action_logp" in extra:
                    ep["pending"] = (obs, req["action"], float(extra["action_logp"]), float(extra.get("vf_preds", 0.0)),
                                     np.asarray(extra.get("action_dist_inputs", []), np.float32))
                else:  # an off-policy action: evaluate it under the current policy
                    lp, v, lg = self._evaluate(obs, req["action"])
                    ep["pending"] = (obs, req["action"], lp, v, lg)
            return {}
        if cmd == LOG_RETURNS:
            with self._cv:
                self._open[req["episode_id"]]["reward"] += float(req["reward"])
            env.log_returns(req["episode_id"], req["reward"], req.get("info"))
            return {}
        if cmd == END_EPISODE:
            eid = req["episode_id"]
            with self._cv:
                self._finish(eid)
            try:
                env.end_episode(eid, np.asarray(req["observation"], np.float32))
            except KeyError:
                pass
            return {}
        if cmd == GET_WORKER_ARGS:
            w = self.worker
            return {"observation_space": _space_dict(w.observation_space), "action_space": _space_dict(w.action_space),
                    "model": w.cfg.get("model") or {}, "weights": _weights_json(w.module)}
        if cmd == GET_WEIGHTS:
            return {"weights": _weights_json(self.worker.module), "version": self.worker.weights_version}
        raise ValueError(f"unknown command {cmd!r}")

    # ------------------------------------------------------------------ policy side
    @torch.no_grad()
    def _evaluate(self, obs, action):
        m = self.worker.module
        with self.worker_lock():
            logits, v = m.forward(torch.as_tensor(obs[None]))
            lp = m.dist(logits).logp(torch.as_tensor(np.asarray([action])))
        return float(lp[0]), float(v[0]), logits[0].numpy()

    def worker_lock(self):
        lk = getattr(self.worker, "_module_lock", None)
        if lk is None:
            lk = self.worker._module_lock = threading.Lock()
        return lk

    def _close_pending(self, eid):
        """A new observation / action arrived for ``eid``: its pending step is complete."""
        ep = self._open.get(eid)
        if ep is None or ep["pending"] is None:
            return
        o, a, lp, v, lg = ep["pending"]
        ep["rows"].append((o, a, lp, v, lg, ep["reward"]))
        ep["reward"] = 0.0
        ep["pending"] = None

    def _finish(self, eid):
        ep = self._open.pop(eid, None)
        if ep is None:
            return
        self._close_pending_ep(ep)
        rows = ep["rows"]
        ret = sum(r[5] for r in rows)
        self._returns.append((float(ret), len(rows)))
        self.episodes_finished += 1
        if rows and ep["train"]:
            self._ready.append(rows)
            self._ready_steps += len(rows)
            self._cv.notify_all()

    @staticmethod
    def _close_pending_ep(ep):
        if ep["pending"] is not None:
            o, a, lp, v, lg = ep["pending"]
            ep["rows"].append((o, a, lp, v, lg, ep["reward"]))
            ep["reward"] = 0.0
            ep["pending"] = None

    def _serving_loop(self):
        """Answer GET_ACTION observations in batches with the runner's current module."""
        while True:
            obs, rew, term, trunc, infos, off = self.base_env.poll(timeout=1.0)
            ask = [eid for eid in obs if not term.get(eid) and eid not in off]
            if not ask:
                continue
            with torch.no_grad(), self.worker_lock():
                m = self.worker.module
                o = torch.as_tensor(np.stack([np.asarray(obs[e], np.float32) for e in ask]))
                a, lp, v, logits = m.forward_exploration(o)
            acts = a.numpy()
            with self._cv:
                for i, eid in enumerate(ask):
                    self._close_pending(eid)
                    if eid in self._open:
                        self._open[eid]["pending"] = (np.asarray(obs[eid], np.float32), acts[i].item(),
                                                      float(lp[i]), float(v[i]), logits[i].numpy())
            self.base_env.send_actions({eid: acts[i].item() for i, eid in enumerate(ask)})

    # ------------------------------------------------------------------ reader side
    def next(self, min_steps: Optional[int] = None) -> SampleBatch:
        need = int(min_steps or self.fragment_length)
        with self._cv:
            self._cv.wait_for(lambda: self._ready_steps >= need)
            eps = list(self._ready)
            self._ready.clear()
            self._ready_steps = 0
        rows = [r for ep in eps for r in ep]
        T = len(rows)
        term = np.zeros(T, bool)
        nvf = np.zeros(T, np.float32)
        eid = np.zeros(T, np.int64)
        i = 0
        for k, ep in enumerate(eps):
            n = len(ep)
            term[i + n - 1] = True
            nvf[i: i + n - 1] = [r[3] for r in ep[1:]]
            eid[i: i + n] = self.episodes_finished * 1000 + k
            i += n
        b = SampleBatch({
            SampleBatch.OBS: np.stack([r[0] for r in rows])[None],
            SampleBatch.ACTIONS: np.asarray([r[1] for r in rows])[None],
            SampleBatch.ACTION_LOGP: np.asarray([r[2] for r in rows], np.float32)[None],
            SampleBatch.VF_PREDS: np.asarray([r[3] for r in rows], np.float32)[None],
            SampleBatch.REWARDS: np.asarray([r[5] for r in rows], np.float32)[None],
            SampleBatch.TERMINATEDS: term[None], SampleBatch.TRUNCATEDS: np.zeros((1, T), bool),
            SampleBatch.NEXT_VF_PREDS: nvf[None], SampleBatch.EPS_ID: eid[None]})
        if all(len(r[4]) for r in rows):
            b[SampleBatch.ACTION_DIST_INPUTS] = np.stack([r[4] for r in rows])[None]
        b.fragment_shape = (1, T)
        return b

    def pop_episode_returns(self):
        out = list(self._returns)
        self._returns.clear()
        return out

    def stop(self):
        self.shutdown()
        self.server_close()


def _space_dict(space):
    from ..utils.spaces import Box, Discrete

    if isinstance(space, Discrete):
        return {"type": "Discrete", "n": int(space.n)}
    if isinstance(space, Box):
        return {"type": "Box", "low": np.asarray(space.low).tolist(), "high": np.asarray(space.high).tolist()}
    raise TypeError(f"unsupported space {space!r}")


def _weights_json(module):
    return {k: v.detach().cpu().numpy().tolist() for k, v in module.state_dict().items()}
