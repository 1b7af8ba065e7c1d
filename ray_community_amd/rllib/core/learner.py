"""Learners and LearnerGroup (reference: ``rllib/core/learner/{learner,learner_group}.py``).

A learner owns the RLModule on its GPU. Its update keeps the whole train batch resident in HBM:
one host->device copy, GAE + advantage standardisation as HIP kernels over the env-major
``[N, T]`` fragments, then the minibatch SGD epochs by device-side index permutation.
With ``num_learners > 1`` every learner is a GPU actor in one RCCL process group and gradients
are all-reduced by the framework's bucketed DDP; the batch is split along the env axis.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ... import ops
from ..policy.sample_batch import SampleBatch
from .learner_api import LearnerAPI, LearnerGroupAPI
from .rl_module import RLModule, make_module


def _device(use_gpu: bool):
    if use_gpu and torch.cuda.is_available():
        idx = os.environ.get("RCA_TRAIN_DEVICE_INDEX")
        return torch.device("cuda", int(idx) if idx is not None else torch.cuda.current_device())
    return torch.device("cpu")


class Learner(LearnerAPI):
    def __init__(self, config: Dict, obs_space, act_space, use_gpu: bool = False):
        self.cfg = config
        self.device = _device(use_gpu)
        seed = config.get("seed")
        if seed is not None:
            torch.manual_seed(int(seed))
        self.module = make_module(config, obs_space, act_space).to(self.device)
        if (self.device.type == "cuda" and config.get("learner_channels_last", True)
                and os.environ.get("RCA_LEARNER_NHWC", "1") != "0"):
            # NHWC conv weights (and NHWC frames from the normalize kernel, RLModule._x): MIOpen's
            # NHWC implicit-GEMM convolutions run without the NCHW<->NHWC batched transposes that
            # were ~10 % of the NatureCNN update's kernel time (scripts/learner_graph_bench.py)
            self.module.to(memory_format=torch.channels_last)
        self.ddp = None
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            from ...parallel import DistributedDataParallel

            self.ddp = DistributedDataParallel(self.module, bucket_cap_mb=64, average_in_optimizer=False,
                                               auto_finalize=True)
            self.ddp.comm_timer.enabled = True  # exposed gradient all-reduce time, per update
        # capturable on the GPU: its step counters live on the device, so the PPO minibatch step
        # (forward, loss, backward, clip, Adam) can be replayed as one HIP graph (_PPOStepGraph)
        self.opt = torch.optim.Adam(self.module.parameters(), lr=config.get("lr", 5e-5),
                                    eps=config.get("adam_epsilon", 1e-8), capturable=self.device.type == "cuda")
        self._ppo_graph = None
        self.kl_coeff = config.get("kl_coeff", 0.2)
        self.target = None
        self.num_updates = 0
        self.last_target_update = 0  # APPO: learner update count at the last target refresh
        self.num_target_updates = 0
        from ..connectors import build_learner_connector

        self.learner_connector = build_learner_connector(config, obs_space, act_space)

    def forward(self, obs, *args):
        return (self.ddp or self.module)(obs, *args)

    def get_weights(self):
        return self.module.get_state()

    def set_weights(self, state):
        self.module.set_state(state)
        self._ppo_graph = None  # a captured step holds the parameter tensors it was recorded with

    def get_state(self):
        st = {"module": self.module.get_state(), "opt": self.opt.state_dict(), "kl_coeff": self.kl_coeff,
              "num_updates": self.num_updates, "last_target_update": self.last_target_update,
              "num_target_updates": self.num_target_updates}
        if self.target is not None:
            st["target"] = {k: v.detach().cpu().clone() for k, v in self.target.state_dict().items()}
        return st

    def set_state(self, st):
        self.module.set_state(st["module"])
        self.opt.load_state_dict(st["opt"])  # new optimizer-state tensors: recapture
        self._ppo_graph = None
        self.kl_coeff = st.get("kl_coeff", self.kl_coeff)
        self.num_updates = st.get("num_updates", self.num_updates)
        self.last_target_update = st.get("last_target_update", self.last_target_update)
        self.num_target_updates = st.get("num_target_updates", self.num_target_updates)
        if "target" in st:
            import copy

            if self.target is None:
                self.target = copy.deepcopy(self.module)
                for p in self.target.parameters():
                    p.requires_grad_(False)
            self.target.load_state_dict({k: v.to(self.device) for k, v in st["target"].items()})

    def _lr(self):
        sched = self.cfg.get("lr_schedule")
        if not sched:
            return self.cfg.get("lr", 5e-5)
        t = self.num_updates
        pts = sorted(sched)
        for (t0, v0), (t1, v1) in zip(pts, pts[1:]):
            if t0 <= t < t1:
                return v0 + (v1 - v0) * (t - t0) / (t1 - t0)
        return pts[-1][1]

    def _step(self, loss):
        if self.ddp is not None:
            # gradients must stay views into DDP's flat buffer (the all-reduce runs on it);
            # set_to_none would make backward allocate detached .grad tensors
            self.ddp.zero_grad()
        else:
            self.opt.zero_grad(set_to_none=True)
        loss.backward()
        gc = self.cfg.get("grad_clip")
        gn = None
        if gc:
            gn = torch.nn.utils.clip_grad_norm_(self.module.parameters(), gc)
        for g in self.opt.param_groups:
            g["lr"] = self._lr()
        self.opt.step()
        return gn

    # ------------------------------------------------------------------ PPO
    def _dist_group(self):
        import torch.distributed as dist

        return self.ddp is not None and dist.is_initialized() and dist.get_world_size() > 1

    def _allreduce_sum(self, t):
        """Sum over the learner group (no-op for a single learner)."""
        if self._dist_group():
            import torch.distributed as dist

            dist.all_reduce(t)
        return t

    def update_ppo(self, batch: SampleBatch) -> Dict:
        """Clipped-surrogate PPO over the batch resident on this learner's device.

        ``loss_mask`` (optional, multi-agent padding): rows with mask 0 carry no loss and are left
        out of the advantage statistics. With several learners the advantage mean/std and the
        reported statistics are reduced over the whole group (each learner holds an env-axis
        shard), so N learners take exactly the step one learner would on the full batch."""
        cfg = self.cfg
        t0 = time.perf_counter()
        b = _to_device_batch(batch, self.device)
        N, T = b.fragment_shape
        if len(self.learner_connector):
            b = self.learner_connector(rl_module=self.module, batch=b, episodes=None, shared_data={})
        rew, vf, nvf = b["rewards"], b["vf_preds"], b["next_vf_preds"]
        term, trunc = b["terminateds"], b["truncateds"]
        done = term | trunc
        gamma, lam = cfg.get("gamma", 0.99), cfg.get("lambda_", 1.0)
        if "advantages" in b and "value_targets" in b:  # a learner connector (GeneralAdvantageEstimation) made them
            adv, vt = b["advantages"].float(), b["value_targets"].float()
        elif cfg.get("use_gae", True):
            adv, vt = ops.compute_gae(rew, vf, term, done, gamma, lam, next_values=nvf, standardize=False)
        else:
            adv, vt = ops.compute_gae(rew, torch.zeros_like(vf), term, done, gamma, 1.0,
                                      next_values=torch.zeros_like(nvf))
            adv = adv - vf
        adv = adv.reshape(-1).contiguous()
        vt = vt.reshape(-1)
        mask = b["loss_mask"].reshape(-1).float() if "loss_mask" in b else None
        if mask is None and not self._dist_group():
            ops.standardize_(adv)
        else:  # masked and/or group-wide statistics
            m = mask if mask is not None else torch.ones_like(adv)
            st = torch.stack([m.sum(), (adv * m).sum(), (adv * adv * m).sum()]).double()
            self._allreduce_sum(st)
            cnt = st[0].clamp(min=1.0)
            mean = st[1] / cnt
            var = (st[2] / cnt - mean * mean).clamp(min=0.0)
            adv = ((adv - mean.float()) / (var.sqrt().float() + 1e-4)) * m
        obs = b["obs"].reshape((N * T,) + tuple(b["obs"].shape[2:]))
        act = b["actions"].reshape((N * T,) + tuple(b["actions"].shape[2:]))
        old_logp = b["action_logp"].reshape(-1)
        old_vf = vf.reshape(-1)
        old_logits = b["action_dist_inputs"].reshape(N * T, -1) if "action_dist_inputs" in b else None
        n = N * T
        mb = min(int(cfg.get("minibatch_size", 128)), n)
        epochs = int(cfg.get("num_epochs", 30))
        clip, vclip = cfg.get("clip_param", 0.3), cfg.get("vf_clip_param", 10.0)
        vf_coeff, ent_coeff = cfg.get("vf_loss_coeff", 1.0), cfg.get("entropy_coeff", 0.0)
        use_kl = cfg.get("use_kl_loss", True) and old_logits is not None
        keys = ["policy_loss", "vf_loss", "entropy", "mean_kl", "total_loss"]
        hp = (clip, vclip, vf_coeff, ent_coeff, use_kl, use_kl and self.kl_coeff > 0)
        count = 0
        gen = torch.Generator(device=self.device)
        gen.manual_seed(1234 + self.num_updates)
        stateful = getattr(self.module, "is_stateful", False)
        graph = None
        if not stateful and self._ppo_graph_ok():
            full = {"obs": obs, "act": act, "olp": old_logp, "adv": adv, "vt": vt, "olg": old_logits, "w": mask}
            key = (n, mb, hp, self.cfg.get("grad_clip"), self._lr(),
                   tuple((k, tuple(v.shape), v.dtype) for k, v in full.items() if v is not None))
            if self._ppo_graph is None or self._ppo_graph.key != key:
                self._ppo_graph = _PPOStepGraph(key, full, mb, self.device)
            graph = self._ppo_graph
            graph.load(full, self.kl_coeff)
            for _ in range(epochs):
                perm = torch.randperm(n, device=self.device, generator=gen)
                for i in range(0, n - mb + 1, mb):
                    graph.step(self, perm[i: i + mb], hp)
                    count += 1
            acc = graph.acc
        else:
            acc = torch.zeros(len(keys), device=self.device)
            kl_t = torch.full((), self.kl_coeff, device=self.device)
            if stateful:
                minibatches = self._recurrent_minibatches(b, N, T, obs, act, old_logp, adv, vt, old_logits, mask,
                                                          mb, epochs, gen)
            else:
                def minibatches():
                    for _ in range(epochs):
                        perm = torch.randperm(n, device=self.device, generator=gen)
                        for i in range(0, n - mb + 1, mb):
                            idx = perm[i: i + mb]
                            logits, v = self.forward(obs[idx])
                            yield (logits, v, act[idx], old_logp[idx], adv[idx], vt[idx],
                                   old_logits[idx] if old_logits is not None else None,
                                   mask[idx] if mask is not None else None)

            for logits, v, act_mb, olp_mb, a_mb, vt_mb, olg_mb, w in minibatches():
                loss, st = self._ppo_loss(logits, v, act_mb, olp_mb, a_mb, vt_mb, olg_mb, w, hp, kl_t)
                self._step(loss)
                acc.add_(st)
                count += 1
        vec = acc.double() / max(count, 1)
        if self._dist_group():  # every learner adapts kl_coeff from the same group-wide KL
            import torch.distributed as dist

            self._allreduce_sum(vec)
            vec = vec / dist.get_world_size()
        out = {k: float(v) for k, v in zip(keys, vec.tolist())}
        if use_kl:
            kt = cfg.get("kl_target", 0.01)
            if out["mean_kl"] > 2.0 * kt:
                self.kl_coeff *= 1.5
            elif out["mean_kl"] < 0.5 * kt:
                self.kl_coeff *= 0.5
        self.num_updates += 1
        ev = 1 - torch.var(vt - old_vf) / (torch.var(vt) + 1e-8)
        out.update({"kl_coeff": self.kl_coeff, "vf_explained_var": float(ev), "num_minibatches": count,
                    "learner_time_s": time.perf_counter() - t0, "cur_lr": self._lr(),
                    "cuda_graph_replays": graph.replays if graph is not None else 0})
        return out

    def _ppo_graph_ok(self) -> bool:
        """The PPO minibatch step runs as a captured HIP graph on a single GPU learner (DDP's
        bucket hooks issue collectives and host-side bookkeeping a graph cannot replay) without
        an lr schedule (its per-step lr would be baked into the graph)."""
        return (self.device.type == "cuda" and self.ddp is None and not self.cfg.get("lr_schedule")
                and bool(self.cfg.get("learner_cuda_graph", True)) and os.environ.get("RCA_LEARNER_GRAPH", "1") != "0"
                and self.opt.param_groups[0].get("capturable", False))

    def _ppo_loss(self, logits, v, act_mb, olp_mb, a_mb, vt_mb, olg_mb, w, hp, kl_t):
        """Clipped-surrogate loss of one minibatch and its 5 statistics (policy_loss, vf_loss,
        entropy, mean_kl, total_loss) as one device vector. ``kl_t``: the KL coefficient as a
        device scalar, so a captured graph reads the current value at replay."""
        clip, vclip, vf_coeff, ent_coeff, use_kl, kl_on = hp

        def mean(x, w):
            return x.mean() if w is None else (x * w).sum() / w.sum().clamp(min=1.0)

        d = self.module.dist(logits)
        lp = d.logp(act_mb)
        ratio = torch.exp(lp - olp_mb)
        surr = torch.min(ratio * a_mb, ratio.clamp(1 - clip, 1 + clip) * a_mb)
        vf_err = (v - vt_mb) ** 2
        vf_loss = vf_err.clamp(0, vclip) if vclip else vf_err
        ent = d.entropy()
        pi_term, vf_term, ent_term = mean(surr, w), mean(vf_loss, w), mean(ent, w)
        loss = -pi_term + vf_coeff * vf_term - ent_coeff * ent_term
        if use_kl:
            kl = mean(self.module.dist(olg_mb).kl(d), w)
            if kl_on:
                loss = loss + kl_t * kl
        else:
            kl = torch.zeros((), device=logits.device)
        return loss, torch.stack([-pi_term, vf_term, ent_term, kl, loss]).detach()

    def _recurrent_minibatches(self, b, N, T, obs, act, old_logp, adv, vt, old_logits, mask, mb, epochs, gen):
        """Recurrent PPO: the ``[N, T]`` fragments are cut into ``max_seq_len`` chunks (the tail
        padded and masked out), each replayed from the state its first step entered with
        (``state_in``) and reset where ``is_first`` marks a new episode inside the chunk.
        Minibatches are ``minibatch_size // max_seq_len`` whole chunks."""
        L = int(self.module.max_seq_len)
        nch = -(-T // L)
        Tp = nch * L
        S = N * nch

        def chunk(x):  # [N * T, ...] -> [S, L, ...] (tail zero-padded)
            x = x.reshape((N, T) + tuple(x.shape[1:]))
            if Tp != T:
                pad = torch.zeros((N, Tp - T) + tuple(x.shape[2:]), dtype=x.dtype, device=x.device)
                x = torch.cat([x, pad], 1)
            return x.reshape((S, L) + tuple(x.shape[2:]))

        valid = torch.ones(N * T, device=self.device) if mask is None else mask.reshape(-1)
        valid_c = chunk(valid)
        obs_c, act_c, olp_c, adv_c, vt_c = (chunk(x) for x in (obs, act, old_logp, adv, vt))
        olg_c = chunk(old_logits) if old_logits is not None else None
        resets = chunk(b["is_first"].bool().reshape(-1))
        state0 = b["state_in"][:, ::L].reshape(S, -1).float()
        mbs = max(1, mb // L)

        def flat(x):
            return x.reshape((-1,) + tuple(x.shape[2:]))

        def gen_mb():
            for _ in range(epochs):
                perm = torch.randperm(S, device=self.device, generator=gen)
                for i in range(0, S - mbs + 1, mbs):
                    idx = perm[i: i + mbs]
                    logits, v = self.forward(obs_c[idx], state0[idx], resets[idx])
                    yield (flat(logits), flat(v), flat(act_c[idx]), flat(olp_c[idx]), flat(adv_c[idx]),
                           flat(vt_c[idx]), flat(olg_c[idx]) if olg_c is not None else None, flat(valid_c[idx]))

        return gen_mb

    # ------------------------------------------------------------------ IMPALA / APPO
    def _vtrace_targets(self, b, N, T, logits, values):
        """V-trace (HIP kernel) with the learner's current policy/values as the target."""
        cfg = self.cfg
        d = self.module.dist(logits)
        act = b["actions"].reshape((N * T,) + tuple(b["actions"].shape[2:]))
        logp = d.logp(act)
        with torch.no_grad():
            v = values.detach().reshape(N, T)
            # V(s_{t+1}): the learner's own value of the next in-fragment state; the runner's bootstrap
            # at episode cuts (terminal / truncated final obs) and at the fragment end.
            done = (b["terminateds"] | b["truncateds"]).bool()
            nv = b["next_vf_preds"].float().clone()
            inner = ~done[:, :-1]
            nv[:, :-1] = torch.where(inner, v[:, 1:], nv[:, :-1])
            log_rhos = (logp.detach() - b["action_logp"].reshape(-1)).reshape(N, T)
            vs, pg = ops.vtrace(log_rhos, b["rewards"].float(), v, nv, b["terminateds"], done,
                                cfg.get("gamma", 0.99), cfg.get("vtrace_clip_rho_threshold", 1.0),
                                cfg.get("vtrace_clip_c_threshold", 1.0), cfg.get("vtrace_clip_pg_rho_threshold", 1.0))
        return d, logp, act, vs.reshape(-1), pg.reshape(-1)

    def update_impala(self, batch: SampleBatch) -> Dict:
        cfg = self.cfg
        t0 = time.perf_counter()
        b = batch.to_device(self.device)
        N, T = batch.fragment_shape
        obs = b["obs"].reshape((N * T,) + tuple(b["obs"].shape[2:]))
        logits, values = self.forward(obs)
        d, logp, act, vs, pg = self._vtrace_targets(b, N, T, logits, values)
        pi_loss = -(logp * pg).mean()
        vf_loss = 0.5 * ((values - vs) ** 2).mean()
        ent = d.entropy().mean()
        loss = pi_loss + cfg.get("vf_loss_coeff", 0.5) * vf_loss - cfg.get("entropy_coeff", 0.01) * ent
        gn = self._step(loss)
        self.num_updates += 1
        gn_t = gn.detach().float().reshape(()) if gn is not None else torch.full((), float("nan"), device=self.device)
        # ONE device->host transfer for every statistic (no per-stat sync)
        pl, vl, en, tl, g = torch.stack([pi_loss.detach(), vf_loss.detach(), ent.detach(), loss.detach(),
                                         gn_t.to(loss.device)]).tolist()
        return {"policy_loss": pl, "vf_loss": vl, "entropy": en, "total_loss": tl, "grad_gnorm": g,
                "learner_time_s": time.perf_counter() - t0, "cur_lr": self._lr()}

    # ---------------------------------------------------------------- APPO target network
    def _appo_target(self):
        """The APPO target policy (reference ``appo_torch_learner._update_module_target_networks``):
        a frozen copy of the module, created equal to it on the first update and then Polyak-updated
        ``target <- tau * online + (1 - tau) * target`` every ``target_update_frequency`` learner
        updates. It is the "old" policy of the surrogate's importance ratio and of the KL term."""
        if self.target is None:
            import copy

            self.target = copy.deepcopy(self.module)
            for p in self.target.parameters():
                p.requires_grad_(False)
            self.last_target_update = self.num_updates
        return self.target

    @torch.no_grad()
    def update_target_network(self, tau: Optional[float] = None):
        tgt = self._appo_target()
        tau = float(self.cfg.get("tau", 1.0) if tau is None else tau)
        for t, o in zip(tgt.state_dict().values(), self.module.state_dict().values()):
            if t.is_floating_point():
                if tau >= 1.0:
                    t.copy_(o)
                else:
                    t.mul_(1.0 - tau).add_(o, alpha=tau)
            else:
                t.copy_(o)
        self.num_target_updates += 1
        self.last_target_update = self.num_updates

    def update_appo(self, batch: SampleBatch) -> Dict:
        """APPO (reference: ``rllib/algorithms/appo/torch/appo_torch_learner.py``): V-trace with the
        TARGET policy as V-trace's target policy, the surrogate ratio
        ``clip(pi_b / pi_target, 0, 2) * pi / pi_b`` clipped PPO-style, the KL term against the target
        policy, and the target network refreshed every ``target_update_frequency`` updates (Polyak
        ``tau``) with the KL coefficient adapted (x1.5 above 2 * kl_target, x0.5 below half of it).
        Statistics are accumulated on the device and read back once per update."""
        cfg = self.cfg
        t0 = time.perf_counter()
        b = batch.to_device(self.device)
        N, T = batch.fragment_shape
        obs = b["obs"].reshape((N * T,) + tuple(b["obs"].shape[2:]))
        act = b["actions"].reshape((N * T,) + tuple(b["actions"].shape[2:]))
        target = self._appo_target()
        behaviour_logp = b["action_logp"].reshape(-1).float()
        with torch.no_grad():
            tgt_logits, _ = target(obs)
            tgt_dist = self.module.dist(tgt_logits)
            tgt_logp = tgt_dist.logp(act)
            is_ratio = torch.clamp(torch.exp(behaviour_logp - tgt_logp), 0.0, 2.0)
        clip = cfg.get("clip_param", 0.4)
        epochs = int(cfg.get("num_epochs", 1))
        use_kl = bool(cfg.get("use_kl_loss", False))
        acc = torch.zeros(5, device=self.device)  # policy, vf, entropy, kl, total
        for _ in range(epochs):
            logits, values = self.forward(obs)
            with torch.no_grad():
                # V-trace corrections toward the target policy (its log-probs as the target policy's)
                v = values.detach().reshape(N, T)
                done = (b["terminateds"] | b["truncateds"]).bool()
                nv = b["next_vf_preds"].float().clone()
                nv[:, :-1] = torch.where(~done[:, :-1], v[:, 1:], nv[:, :-1])
                log_rhos = (tgt_logp - behaviour_logp).reshape(N, T)
                vs, pg = ops.vtrace(log_rhos, b["rewards"].float(), v, nv, b["terminateds"], done,
                                    cfg.get("gamma", 0.99), cfg.get("vtrace_clip_rho_threshold", 1.0),
                                    cfg.get("vtrace_clip_c_threshold", 1.0),
                                    cfg.get("vtrace_clip_pg_rho_threshold", 1.0))
                vs, pg = vs.reshape(-1), pg.reshape(-1)
            d = self.module.dist(logits)
            logp_ratio = is_ratio * torch.exp(d.logp(act) - behaviour_logp)
            surr = torch.minimum(pg * logp_ratio, pg * torch.clamp(logp_ratio, 1 - clip, 1 + clip))
            vf_loss = 0.5 * ((values - vs) ** 2).mean()
            ent = d.entropy().mean()
            pi_loss = -surr.mean()
            loss = pi_loss + cfg.get("vf_loss_coeff", 0.5) * vf_loss - cfg.get("entropy_coeff", 0.01) * ent
            kl = tgt_dist.kl(d).mean() if use_kl else torch.zeros((), device=self.device)
            if use_kl:
                loss = loss + self.kl_coeff * kl
            self._step(loss)
            acc += torch.stack([pi_loss.detach(), vf_loss.detach(), ent.detach(), kl.detach(), loss.detach()])
        pl, vl, en, klv, tl = (acc / max(epochs, 1)).tolist()  # the update's one host sync
        self.num_updates += 1
        freq = max(1, int(cfg.get("target_update_frequency", 1)))
        updated = 0
        if self.num_updates - self.last_target_update >= freq:
            self.update_target_network()
            updated = 1
            if use_kl:
                kt = cfg.get("kl_target", 0.01)
                if klv > 2.0 * kt:
                    self.kl_coeff *= 1.5
                elif klv < 0.5 * kt:
                    self.kl_coeff *= 0.5
        return {"policy_loss": pl, "vf_loss": vl, "entropy": en, "mean_kl": klv, "total_loss": tl,
                "learner_time_s": time.perf_counter() - t0, "cur_lr": self._lr(), "kl_coeff": self.kl_coeff,
                "num_target_updates": self.num_target_updates, "target_updated": updated,
                "last_target_update": self.last_target_update}

    # ------------------------------------------------------------------ DQN
    def update_dqn(self, batch: SampleBatch) -> Dict:
        cfg = self.cfg
        if self.target is None:
            import copy

            self.target = copy.deepcopy(self.module)
        b = batch.to_device(self.device)
        q = self.module.q_values(b["obs"])
        qa = q.gather(1, b["actions"].long().unsqueeze(1)).squeeze(1)
        with torch.no_grad():
            qn_t = self.target.q_values(b["new_obs"])
            if cfg.get("double_q", True):
                an = self.module.q_values(b["new_obs"]).argmax(1, keepdim=True)
                qn = qn_t.gather(1, an).squeeze(1)
            else:
                qn = qn_t.max(1).values
            # episode replay gives each sample's own step count (n-step returns clipped at the
            # episode's end); the transition buffer uses the configured n_step for all
            n = b["n_step"].float() if "n_step" in b else float(cfg.get("n_step", 1))
            y = b["rewards"] + cfg.get("gamma", 0.99) ** n * (1 - b["terminateds"].float()) * qn
        td = qa - y
        loss = torch.nn.functional.huber_loss(qa, y, delta=1.0) if cfg.get("td_error_loss_fn", "huber") == "huber" \
            else (td ** 2).mean()
        self._step(loss)
        self.num_updates += 1
        return {"loss": loss.item(), "mean_q": qa.mean().item(), "mean_td_error": td.abs().mean().item()}

    # ------------------------------------------------------------------ MARWIL / BC
    def update_marwil(self, batch: SampleBatch) -> Dict:
        cfg = self.cfg
        b = batch.to_device(self.device)
        if batch.fragment_shape is not None:
            N, T = batch.fragment_shape
            rew = b["rewards"].float()
            term, trunc = b["terminateds"].bool(), b["truncateds"].bool()
            nv = torch.zeros_like(rew)
            if "next_vf_preds" in b:
                boot = b["next_vf_preds"].float()
                nv[:, -1] = boot[:, -1]
                nv = torch.where(trunc, boot, nv)
            ret, _ = ops.compute_gae(rew, torch.zeros_like(rew), term, term | trunc, cfg.get("gamma", 0.99), 1.0,
                                     next_values=nv)
            obs = b["obs"].reshape((N * T,) + tuple(b["obs"].shape[2:]))
            act = b["actions"].reshape((N * T,) + tuple(b["actions"].shape[2:]))
            ret = ret.reshape(-1)
        else:
            obs, act = b["obs"], b["actions"]
            ret = b["returns"].float() if "returns" in b else b["rewards"].float()
        logits, v = self.forward(obs)
        logp = self.module.dist(logits).logp(act)
        beta = float(cfg.get("beta", 1.0))
        if beta > 0:
            adv = (ret - v).detach()
            if not hasattr(self, "_adv_c2"):
                self._adv_c2 = float(cfg.get("moving_average_sqd_adv_norm_start", 100.0))
            rate = float(cfg.get("moving_average_sqd_adv_norm_update_rate", 1e-8))
            self._adv_c2 += rate * (float((adv ** 2).mean()) - self._adv_c2)
            w = torch.exp(beta * adv / (self._adv_c2 ** 0.5 + 1e-8)).clamp(max=20.0)
        else:
            w = torch.ones_like(logp)
        pi_loss = -(w * logp).mean()
        vf_loss = 0.5 * ((ret - v) ** 2).mean()
        loss = pi_loss + float(cfg.get("vf_coeff", 1.0)) * vf_loss
        self._step(loss)
        self.num_updates += 1
        return {"policy_loss": pi_loss.item(), "vf_loss": vf_loss.item(), "total_loss": loss.item(),
                "mean_logp": logp.detach().mean().item()}

    # ------------------------------------------------------------------ SAC
    def update_sac(self, batch: SampleBatch) -> Dict:
        """Twin-Q soft actor-critic step (reference: rllib/algorithms/sac/torch/sac_torch_learner.py)."""
        cfg = self.cfg
        m = self.module
        if not hasattr(self, "_sac_opts"):
            lr = cfg.get("lr", 3e-4)
            olr = cfg.get("optimization_config") or {}
            self._sac_opts = (
                torch.optim.Adam(m.pi.parameters(), lr=olr.get("actor_learning_rate", lr)),
                torch.optim.Adam(list(m.q1.parameters()) + list(m.q2.parameters()),
                                 lr=olr.get("critic_learning_rate", lr)),
                torch.optim.Adam([m.log_alpha], lr=olr.get("entropy_learning_rate", lr)))
            te = cfg.get("target_entropy", "auto")
            self._target_entropy = -float(m.act_dim) if te in (None, "auto") else float(te)
        opt_pi, opt_q, opt_a = self._sac_opts
        b = batch.to_device(self.device)
        obs, nobs = b["obs"].float(), b["new_obs"].float()
        u = m._unscale(b["actions"].float().reshape(obs.shape[0], -1))
        r, term = b["rewards"].float(), b["terminateds"].float()
        gamma = cfg.get("gamma", 0.99) ** cfg.get("n_step", 1)
        alpha = m.log_alpha.exp().detach()
        with torch.no_grad():
            un, lpn = m.policy(nobs)
            q1t, q2t = m.q(nobs, un, target=True)
            y = r + gamma * (1 - term) * (torch.min(q1t, q2t) - alpha * lpn)
        q1, q2 = m.q(obs, u)
        q_loss = 0.5 * (((q1 - y) ** 2).mean() + ((q2 - y) ** 2).mean())
        opt_q.zero_grad(set_to_none=True)
        q_loss.backward()
        gc = cfg.get("grad_clip")
        if gc:
            torch.nn.utils.clip_grad_norm_(list(m.q1.parameters()) + list(m.q2.parameters()), gc)
        opt_q.step()
        un, lp = m.policy(obs)
        q1n, q2n = m.q(obs, un)
        pi_loss = (alpha * lp - torch.min(q1n, q2n)).mean()
        opt_pi.zero_grad(set_to_none=True)
        pi_loss.backward()
        opt_pi.step()
        a_loss = -(m.log_alpha * (lp.detach() + self._target_entropy)).mean()
        opt_a.zero_grad(set_to_none=True)
        a_loss.backward()
        opt_a.step()
        m.polyak(cfg.get("tau", 5e-3))
        self.num_updates += 1
        return {"critic_loss": q_loss.item(), "actor_loss": pi_loss.item(), "alpha_loss": a_loss.item(),
                "alpha_value": alpha.item(), "mean_q": q1.detach().mean().item()}

    # ------------------------------------------------------------------ CQL
    def update_cql(self, batch: SampleBatch) -> Dict:
        """Conservative Q-learning step (reference: rllib/algorithms/cql/cql_torch_policy.py): the
        SAC losses plus, per critic, ``min_q_weight * (T * logsumexp(Q(s, a~{uniform, pi(s),
        pi(s')}) / T - log-density) - Q(s, a_data))``; optional Lagrangian weight tuned to
        ``lagrangian_thresh``; the actor clones the logged actions for the first ``bc_iters``
        updates."""
        cfg = self.cfg
        m = self.module
        if not hasattr(self, "_cql_opts"):
            lr = cfg.get("lr", 3e-4)
            olr = cfg.get("optimization_config") or {}
            self._log_alpha_prime = torch.zeros((), device=self.device, requires_grad=True)
            self._cql_opts = (
                torch.optim.Adam(m.pi.parameters(), lr=olr.get("actor_learning_rate", lr)),
                torch.optim.Adam(list(m.q1.parameters()) + list(m.q2.parameters()),
                                 lr=olr.get("critic_learning_rate", lr)),
                torch.optim.Adam([m.log_alpha], lr=olr.get("entropy_learning_rate", lr)),
                torch.optim.Adam([self._log_alpha_prime], lr=olr.get("critic_learning_rate", lr)))
            te = cfg.get("target_entropy", "auto")
            self._target_entropy = -float(m.act_dim) if te in (None, "auto") else float(te)
        opt_pi, opt_q, opt_a, opt_ap = self._cql_opts
        b = batch.to_device(self.device)
        obs, nobs = b["obs"].float(), b["new_obs"].float()
        B = obs.shape[0]
        u = m._unscale(b["actions"].float().reshape(B, -1)).clamp(-1.0, 1.0)
        r, term = b["rewards"].float(), b["terminateds"].float()
        gamma = cfg.get("gamma", 0.99) ** cfg.get("n_step", 1)
        alpha = m.log_alpha.exp().detach()
        K = int(cfg.get("num_actions", 10))
        T = float(cfg.get("temperature", 1.0))
        wq = float(cfg.get("min_q_weight", 5.0))
        with torch.no_grad():
            un, lpn = m.policy(nobs)
            q1t, q2t = m.q(nobs, un, target=True)
            y = r + gamma * (1 - term) * (torch.min(q1t, q2t) - alpha * lpn)
            # the CQL action samples: uniform on [-1, 1]^A (log-density -A log 2), pi(.|s), pi(.|s')
            obs_k = obs.repeat_interleave(K, 0)
            nobs_k = nobs.repeat_interleave(K, 0)
            u_rand = torch.rand(B * K, m.act_dim, device=obs.device) * 2 - 1
            u_cur, lp_cur = m.policy(obs_k)
            u_nxt, lp_nxt = m.policy(nobs_k)
            lp_rand = -m.act_dim * math.log(2.0)
        q1, q2 = m.q(obs, u)
        bellman = 0.5 * (((q1 - y) ** 2).mean() + ((q2 - y) ** 2).mean())
        xs = torch.cat([obs_k, obs_k, obs_k], 0)
        us = torch.cat([u_rand, u_cur, u_nxt], 0)
        dens = torch.cat([torch.full((B * K,), lp_rand, device=obs.device), lp_cur, lp_nxt], 0)
        qs1, qs2 = m.q(xs, us)
        pen = []
        for qs, qd in ((qs1, q1), (qs2, q2)):
            cat = (qs - dens).view(3, B, K).permute(1, 0, 2).reshape(B, 3 * K)
            pen.append(wq * (T * torch.logsumexp(cat / T, dim=1).mean() - qd.mean()))
        info = {}
        if cfg.get("lagrangian", False):
            ap = self._log_alpha_prime.exp().clamp(0.0, 1e6)
            thresh = float(cfg.get("lagrangian_thresh", 5.0))
            ap_loss = -0.5 * ap * ((pen[0].detach() - thresh) + (pen[1].detach() - thresh))
            pen = [ap.detach() * (p - thresh) for p in pen]
            opt_ap.zero_grad(set_to_none=True)
            ap_loss.backward()
            opt_ap.step()
            info["alpha_prime_value"] = ap.item()
        q_loss = bellman + pen[0] + pen[1]
        opt_q.zero_grad(set_to_none=True)
        q_loss.backward()
        gc = cfg.get("grad_clip")
        if gc:
            torch.nn.utils.clip_grad_norm_(list(m.q1.parameters()) + list(m.q2.parameters()), gc)
        opt_q.step()
        un, lp = m.policy(obs)
        if self.num_updates < int(cfg.get("bc_iters", 20000)):
            pi_loss = (alpha * lp - m.logp_of(obs, u)).mean()
        else:
            q1n, q2n = m.q(obs, un)
            pi_loss = (alpha * lp - torch.min(q1n, q2n)).mean()
        opt_pi.zero_grad(set_to_none=True)
        pi_loss.backward()
        opt_pi.step()
        a_loss = -(m.log_alpha * (lp.detach() + self._target_entropy)).mean()
        opt_a.zero_grad(set_to_none=True)
        a_loss.backward()
        opt_a.step()
        m.polyak(cfg.get("tau", 5e-3))
        self.num_updates += 1
        info.update({"critic_loss": q_loss.item(), "bellman_loss": bellman.item(), "cql_loss": (pen[0] + pen[1]).item(),
                     "actor_loss": pi_loss.item(), "alpha_loss": a_loss.item(), "alpha_value": alpha.item(),
                     "mean_q": q1.detach().mean().item()})
        return info

    def sync_target(self):
        if self.target is not None:
            self.target.load_state_dict(self.module.state_dict())


class _PPOStepGraph:
    """One PPO minibatch step -- gather the minibatch rows by index, forward, loss, backward,
    gradient clipping, capturable Adam, statistics accumulation -- captured once as a HIP graph
    (``torch.cuda.CUDAGraph``) and replayed for every later minibatch with the same shapes.

    The eager step is launch-bound at RLlib sizes (~150 small kernels, each a Python dispatch);
    a replay is one graph launch. The whole train batch lives in static device buffers (one copy
    per update), the minibatch is selected by a static index buffer (the device permutation's
    slice, copied in before each replay), the KL coefficient is a device scalar, and the running
    statistics are a device vector the graph adds into. The first ``WARM`` minibatches run eagerly
    on a side stream (autograd / MIOpen / Adam-state initialisation must happen outside the
    capture; they are real training steps), the next is captured and replayed. The replayed
    kernels are the eager ones, so the path is bitwise equal to the eager loop
    (tests/test_rllib_learner_graph_gpu.py)."""

    WARM = 2

    def __init__(self, key, full, mb, device):
        self.key = key
        self.device = device
        self.full = {k: torch.empty_like(v) for k, v in full.items() if v is not None}
        self.idx = torch.zeros(mb, dtype=torch.long, device=device)
        self.kl_t = torch.zeros((), device=device)
        self.acc = torch.zeros(5, device=device)
        self.graph = None
        self.warm = 0
        self.replays = 0

    def load(self, full, kl_coeff):
        for k, v in full.items():
            if v is not None:
                self.full[k].copy_(v)
        self.kl_t.fill_(kl_coeff)
        self.acc.zero_()
        self.replays = 0

    def _body(self, lr):
        f, idx = self.full, self.idx
        g = lambda k: f[k][idx] if k in f else None  # noqa: E731
        logits, v = lr.forward(g("obs"))
        loss, st = lr._ppo_loss(logits, v, g("act"), g("olp"), g("adv"), g("vt"), g("olg"), g("w"), self._hp,
                                self.kl_t)
        lr._step(loss)
        self.acc.add_(st)

    def step(self, lr, idx, hp):
        self._hp = hp
        self.idx.copy_(idx)
        if self.graph is not None:
            self.graph.replay()
            self.replays += 1
            return
        cur = torch.cuda.current_stream(self.device)
        if self.warm < self.WARM:
            side = torch.cuda.Stream(self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._body(lr)
            cur.wait_stream(side)
            self.warm += 1
            return
        lr.opt.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self._body(lr)
        self.graph = graph
        graph.replay()  # the capture recorded this minibatch's step without running it
        self.replays += 1


def _learner_actor_cls():
    from ...train._internal.worker_group import _TrainWorker

    class _LearnerActor(_TrainWorker):
        """A Train worker (node info, process-group setup via the torch backend) hosting a Learner."""

        def __init__(self):
            super().__init__()
            self.learner = None

        def build(self, config, obs_space, act_space, use_gpu):
            self.learner = Learner(config, obs_space, act_space, use_gpu)
            return True

        def update(self, kind, batch):
            t0 = time.perf_counter()
            if isinstance(batch, (list, tuple)) and batch and not isinstance(batch[0], SampleBatch):
                batch = self._fetch_fragments(list(batch))
            out = getattr(self.learner, f"update_{kind}")(batch)
            out = dict(out)
            out["rank_update_time_s"] = time.perf_counter() - t0
            ddp = self.learner.ddp
            out["exposed_comm_ms"] = ddp.comm_timer.take_ms() if ddp is not None else 0.0
            return out

        def call(self, name, *args):
            return getattr(self.learner, name)(*args)

        def _fetch_fragments(self, refs):
            """Runner fragments by reference: each is mapped from the shared-memory store and copied
            to this learner's device the moment its runner finishes, while the others still
            sample (in fragment order in the result)."""
            from ..._private.worker import get, wait

            pos = {r: i for i, r in enumerate(refs)}
            out = [None] * len(refs)
            pending = list(refs)
            dev = self.learner.device
            while pending:
                ready, pending = wait(pending, num_returns=1)
                for r in ready:
                    fr = get(r)
                    out[pos[r]] = fr.to_device(dev) if dev.type == "cuda" else fr
            return out

    return _LearnerActor


class LearnerGroup(LearnerGroupAPI):
    """``num_learners == 0``: one local learner in the driver (on a GPU if the driver has one).
    ``num_learners >= 1``: GPU learner actors in a placement group, one RCCL process group."""

    def __init__(self, config: Dict, obs_space, act_space):
        self.cfg = config
        self.n = int(config.get("num_learners", 0))
        gpus = float(config.get("num_gpus_per_learner", 0) or 0)
        self.use_gpu = gpus > 0 or (self.n == 0 and config.get("num_gpus", 0) > 0)
        if self.n == 0:
            self.local = Learner(config, obs_space, act_space, self.use_gpu)
            self.wg = None
            return
        from ...train._internal.worker_group import WorkerGroup
        from ...train.torch.config import TorchConfig, _TorchBackend
        from ...air.config import ScalingConfig
        from ..._private.worker import get

        res = {"CPU": 1, "GPU": gpus} if gpus else {"CPU": 1}
        self.wg = WorkerGroup(self.n, res, "PACK", actor_cls=_learner_actor_cls())
        sc = ScalingConfig(num_workers=self.n, use_gpu=gpus > 0, resources_per_worker=res)
        _TorchBackend().on_start(self.wg, TorchConfig(), sc)
        get([w.build.remote(config, obs_space, act_space, gpus > 0) for w in self.wg.workers])
        self.local = None

    def update(self, kind: str, batch: SampleBatch) -> Dict:
        if self.local is not None:
            return getattr(self.local, f"update_{kind}")(batch)
        from ..._private.worker import get

        shards = _split(batch, self.n)
        res = get([w.update.remote(kind, s) for w, s in zip(self.wg.workers, shards)])
        out = {}
        for k in res[0]:
            vals = [r[k] for r in res if isinstance(r.get(k), (int, float))]
            if vals:
                out[k] = float(np.mean(vals))
        # per-rank timings: the slowest learner sets the update's time; exposed_comm_ms is each
        # rank's wait on the gradient all-reduce (what overlap with backward did not hide)
        out["rank_update_time_s"] = [float(r.get("rank_update_time_s", 0.0)) for r in res]
        out["rank_exposed_comm_ms"] = [float(r.get("exposed_comm_ms", 0.0)) for r in res]
        out["exposed_comm_ms"] = max(out["rank_exposed_comm_ms"])
        return out

    def call(self, name, *args):
        if self.local is not None:
            return getattr(self.local, name)(*args)
        from ..._private.worker import get

        return get([w.call.remote(name, *args) for w in self.wg.workers])[0]

    def get_weights(self):
        return self.call("get_weights")

    def shutdown(self):
        if self.wg is not None:
            self.wg.shutdown()


def _to_device_batch(batch, device) -> SampleBatch:
    """One device-resident train batch. A list of runner fragments is copied host->device
    fragment by fragment and stacked ON THE DEVICE (``concat_samples`` -> HIP ``batched_concat``,
    one launch per column), so the driver never concatenates the rollouts on the host."""
    if isinstance(batch, (list, tuple)):
        from ..policy.sample_batch import concat_samples

        return concat_samples([b.to_device(device) for b in batch if b is not None and b.count > 0])
    return batch.to_device(device)


def _split(batch, n: int) -> List:
    if isinstance(batch, (list, tuple)):
        if len(batch) >= n and len(batch) % n == 0:  # whole runner fragments per learner
            k = len(batch) // n
            return [list(batch[i * k: (i + 1) * k]) for i in range(n)]
        from ..policy.sample_batch import concat_samples

        batch = concat_samples(list(batch))
    if batch.fragment_shape is not None:
        N, T = batch.fragment_shape
        per = [N // n + (1 if i < N % n else 0) for i in range(n)]
        outs, s = [], 0
        for p in per:
            sb = SampleBatch({k: v[s: s + p] for k, v in batch.items()})
            sb.fragment_shape = (p, T)
            outs.append(sb)
            s += p
        return outs
    c = batch.count
    per = math.ceil(c / n)
    return [batch.slice(i * per, min(c, (i + 1) * per)) for i in range(n)]
