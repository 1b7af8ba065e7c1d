"""External simulators over HTTP, client side (reference: ``rllib/env/policy_client.py:58``).

A simulator that cannot be wrapped as an env (it runs elsewhere, owns its own loop) drives
training through a ``PolicyClient`` connected to a ``PolicyServerInput``:

    client = PolicyClient("http://127.0.0.1:9900", inference_mode="local")
    eid = client.start_episode()
    obs = sim.reset()
    while not done:
        action = client.get_action(eid, obs)
        obs, reward, done = sim.step(action)
        client.log_returns(eid, reward)
    client.end_episode(eid, obs)

``inference_mode="remote"``: every ``get_action`` is a round trip; the server's current policy
answers. ``"local"``: the client keeps a copy of the policy (spaces, model config and weights
fetched from the server, refreshed every ``update_interval`` seconds), acts on it locally and
logs the action with the policy outputs PPO's loss needs (``action_logp``, ``vf_preds``,
``action_dist_inputs``).
"""
from __future__ import annotations

import json
import time
import urllib.request
from typing import Any, Dict, Optional

import numpy as np
import torch

from .policy_server_input import (END_EPISODE, GET_ACTION, GET_WEIGHTS, GET_WORKER_ARGS, LOG_ACTION, LOG_RETURNS,
                                  START_EPISODE, _jsonable)


class PolicyClient:
    def __init__(self, address: str, inference_mode: str = "local", update_interval: Optional[float] = 10.0,
                 timeout: float = 60.0):
        if inference_mode not in ("local", "remote"):
            raise ValueError("inference_mode must be 'local' or 'remote'")
        self.address = address if address.startswith("http") else f"http://{address}"
        self.inference_mode = inference_mode
        self.update_interval = update_interval
        self.timeout = timeout
        self.module = None
        self._last_update = 0.0
        if inference_mode == "local":
            self._setup_local()

    # ------------------------------------------------------------------ transport
    def _send(self, req: Dict) -> Dict:
        data = json.dumps(_jsonable(req)).encode()
        r = urllib.request.Request(self.address, data=data, headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(r, timeout=self.timeout) as resp:
                out = json.loads(resp.read().decode())
        except urllib.error.HTTPError as e:
            raise RuntimeError(json.loads(e.read().decode()).get("error", str(e))) from None
        return out

    # ------------------------------------------------------------------ local policy copy
    def _setup_local(self):
        from ..core.rl_module import make_module
        from ..utils.spaces import Box, Discrete

        args = self._send({"command": GET_WORKER_ARGS})

        def space(d):
            if d["type"] == "Discrete":
                return Discrete(d["n"])
            return Box(np.asarray(d["low"], np.float32), np.asarray(d["high"], np.float32), dtype=np.float32)

        self.module = make_module({"model": args["model"]}, space(args["observation_space"]),
                                  space(args["action_space"]))
        self.module.eval()
        self._load(args["weights"])

    def _load(self, weights: Dict[str, Any]):
        self.module.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in weights.items()})
        self._last_update = time.time()

    def update_policy_weights(self):
        """Pull the server's current weights into the local policy copy."""
        if self.module is not None:
            self._load(self._send({"command": GET_WEIGHTS})["weights"])

    def _maybe_update(self):
        if self.update_interval is not None and time.time() - self._last_update > self.update_interval:
            self.update_policy_weights()

    # ------------------------------------------------------------------ episode API
    def start_episode(self, episode_id: Optional[str] = None, training_enabled: bool = True) -> str:
        return self._send({"command": START_EPISODE, "episode_id": episode_id,
                           "training_enabled": training_enabled})["episode_id"]

    def get_action(self, episode_id: str, observation):
        if self.inference_mode == "remote":
            a = self._send({"command": GET_ACTION, "episode_id": episode_id, "observation": observation})["action"]
            return a
        self._maybe_update()
        with torch.no_grad():
            o = torch.as_tensor(np.asarray(observation, np.float32)[None])
            a, lp, v, logits = self.module.forward_exploration(o)
        act = a[0].numpy()
        act = act.item() if act.ndim == 0 else act
        self._send({"command": LOG_ACTION, "episode_id": episode_id, "observation": observation, "action": act,
                    "extra": {"action_logp": float(lp[0]), "vf_preds": float(v[0]),
                              "action_dist_inputs": logits[0].numpy()}})
        return act

    def log_action(self, episode_id: str, observation, action):
        """The simulator chose ``action`` itself (off-policy): the server evaluates it under the
        current policy for the training batch."""
        self._send({"command": LOG_ACTION, "episode_id": episode_id, "observation": observation, "action": action})

    def log_returns(self, episode_id: str, reward: float, info: Optional[Dict] = None, multiagent_done_dict=None):
        self._send({"command": LOG_RETURNS, "episode_id": episode_id, "reward": float(reward), "info": info})

    def end_episode(self, episode_id: str, observation):
        self._send({"command": END_EPISODE, "episode_id": episode_id, "observation": observation})
