"""Torch-CPU restatement of the reference train step -- TEST / MEASUREMENT INFRASTRUCTURE ONLY.

``bench.py``'s ``cpu_baseline`` times this on the GPU box's host cores ("CPU
baseline timing" (2): the reference's own Python cannot travel to the box, so a from-scratch
torch-CPU restatement of the same computation, parity-checked here against the reference's
goldens by ``tests/test_torch_cpu_restatement.py``, stands in for it).  It computes what the
reference's CPU path computes, with the same library calls on the hot path: ``F.linear`` /
``F.relu`` / ``F.layer_norm`` forward, autograd backward, ``torch.optim.Adam`` (CPU:
single-tensor, ``torch/optim/adam.py:347``) and the in-place Polyak update.  Nothing in
``td3_amd/`` imports it.

* ``FeaturedTorch``: ``TD3_featured.TD3.train`` (TD3_featured.py:123-171), Actor / Q
  (:15-96; ReLU then LayerNorm, eps 1e-5; ``max_action * tanh`` policy; twin critic).
* ``ParticleTorch``: ``TD3_particles.TD3.train`` / ``_actor_learn`` (TD3_particles.py:167-224):
  the per-particle encoder conv1 (1 x D) -> ReLU -> conv2 (1 x 1) -> ReLU -> mean over the
  particles -> ReLU (:52-58, written as the equivalent matmuls over [B, N, D]), ``lnorm1`` on
  ``[pooled, features(, action)]``, Q heads with one output per action, no clamp of the smoothed
  target action, ``tanh`` policy, CDQ optional.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _params(d):
    return {k: torch.tensor(np.asarray(v, dtype=np.float32)).requires_grad_(True) for k, v in d.items()}


def _copy(d):
    return {k: v.detach().clone() for k, v in d.items()}


def _mlp(P, prefix, x, norm):
    """linears.{0..2} with ReLU then LayerNorm, linears.3 plain (TD3_featured.py:39-48, :73-81)."""
    for i in range(3):
        x = F.relu(F.linear(x, P[f"{prefix}linears.{i}.weight"], P[f"{prefix}linears.{i}.bias"]))
        if norm == "layer":
            x = F.layer_norm(x, (x.shape[1],), P[f"{prefix}lnorms.{i}.weight"], P[f"{prefix}lnorms.{i}.bias"], 1e-5)
    return F.linear(x, P[f"{prefix}linears.3.weight"], P[f"{prefix}linears.3.bias"])


class _Base:
    def __init__(self, actor, critic, *, max_action=1.0, discount=0.99, tau=0.005, policy_noise=0.2,
                 noise_clip=0.5, policy_freq=2, lr=1e-4, norm="layer", cdq=True):
        if norm not in ("layer", None):
            raise ValueError("the torch-CPU restatement covers norm='layer' and None")
        self.A, self.C = _params(actor), _params(critic)
        self.AT, self.CT = _copy(self.A), _copy(self.C)               # deepcopy (TD3_featured.py:102,107)
        self.aopt = torch.optim.Adam(list(self.A.values()), lr=lr, foreach=False)
        self.copt = torch.optim.Adam(list(self.C.values()), lr=lr, foreach=False)
        self.max_action, self.discount, self.tau = max_action, discount, tau
        self.policy_noise, self.noise_clip, self.policy_freq = policy_noise, noise_clip, policy_freq
        self.norm, self.cdq = norm, cdq
        self.total_it = 0

    def _polyak(self):                                                # TD3_featured.py:167-171
        with torch.no_grad():
            for src, dst in ((self.C, self.CT), (self.A, self.AT)):
                for k in src:
                    dst[k].copy_(self.tau * src[k] + (1 - self.tau) * dst[k])

    def numpy(self, which):
        d = {"actor": self.A, "critic": self.C, "actor_target": self.AT, "critic_target": self.CT}[which]
        return {k: v.detach().numpy().copy() for k, v in d.items()}


class FeaturedTorch(_Base):
    def actor(self, P, s):
        return self.max_action * torch.tanh(_mlp(P, "", s, self.norm))

    def q(self, P, prefix, s, a):
        return _mlp(P, prefix, torch.cat([s, a], 1), self.norm)       # TD3_featured.py:74

    def train_step(self, batch, noise):
        """One TD3_featured.TD3.train on a gathered fp32 batch; noise = the randn_like draw."""
        s, a, s2, r, nd = (torch.from_numpy(np.asarray(x, dtype=np.float32)) for x in batch)
        self.total_it += 1
        with torch.no_grad():                                         # :129-142
            eps = (torch.from_numpy(np.asarray(noise, np.float32)) * self.policy_noise).clamp(
                -self.noise_clip, self.noise_clip)
            na = (self.actor(self.AT, s2) + eps).clamp(-self.max_action, self.max_action)
            tq = torch.min(self.q(self.CT, "q1.", s2, na), self.q(self.CT, "q2.", s2, na))
            y = r + nd * self.discount * tq
        q1, q2 = self.q(self.C, "q1.", s, a), self.q(self.C, "q2.", s, a)
        loss = F.mse_loss(q1, y) + F.mse_loss(q2, y)                  # :148
        self.copt.zero_grad()
        loss.backward()
        self.copt.step()
        rec = {"y": y.numpy(), "q1": q1.detach().numpy(), "q2": q2.detach().numpy(), "critic_loss": float(loss.detach())}
        if self.total_it % self.policy_freq == 0:                      # :156-171
            al = -self.q(self.C, "q1.", s, self.actor(self.A, s)).mean()
            self.aopt.zero_grad()
            al.backward()
            self.aopt.step()
            self._polyak()
            rec["actor_loss"] = float(al.detach())
        return rec


class ParticleTorch(_Base):
    def _net(self, P, prefix, f, p, a=None):
        W1 = P[f"{prefix}conv1.weight"].reshape(P[f"{prefix}conv1.weight"].shape[0], -1)   # [256, D]
        W2 = P[f"{prefix}conv2.weight"][:, :, 0]                                           # [128, 256]
        h = F.relu(F.linear(p, W1, P[f"{prefix}conv1.bias"]))        # conv1 (1 x D)  [B, N, 256]
        h = F.relu(F.linear(h, W2, P[f"{prefix}conv2.bias"]))        # conv2 (1 x 1)  [B, N, 128]
        x = torch.cat([F.relu(h.mean(1)), f] + ([a] if a is not None else []), 1)   # :52-59 / :103-110
        if self.norm == "layer":
            x = F.layer_norm(x, (x.shape[1],), P[f"{prefix}lnorm1.weight"], P[f"{prefix}lnorm1.bias"], 1e-5)
        return _mlp(P, prefix, x, self.norm)

    def actor(self, P, f, p):
        return torch.tanh(self._net(P, "", f, p))                      # :68 (no max_action)

    def train_step(self, batch, noise):
        f, p, a, f2, p2, r, nd = (torch.from_numpy(np.asarray(x, dtype=np.float32)) for x in batch)
        self.total_it += 1
        with torch.no_grad():                                         # :173-189
            eps = (torch.from_numpy(np.asarray(noise, np.float32)) * self.policy_noise).clamp(
                -self.noise_clip, self.noise_clip)
            na = self.actor(self.AT, f2, p2) + eps                     # no clamp (:179-181)
            tq = self._net(self.CT, "q1.", f2, p2, na)
            if self.cdq:
                tq = torch.min(tq, self._net(self.CT, "q2.", f2, p2, na))
            y = r + nd * self.discount * tq
        q1 = self._net(self.C, "q1.", f, p, a)
        loss = F.mse_loss(q1, y)
        rec = {"y": y.numpy(), "q1": q1.detach().numpy()}
        if self.cdq:
            q2 = self._net(self.C, "q2.", f, p, a)
            loss = loss + F.mse_loss(q2, y)
            rec["q2"] = q2.detach().numpy()
        self.copt.zero_grad()
        loss.backward()
        self.copt.step()
        rec["critic_loss"] = float(loss.detach())
        if self.total_it % self.policy_freq == 0:
            rec["actor_loss"] = self.actor_learn(f, p)
        return rec

    def actor_learn(self, f, p):                                       # _actor_learn, :209-224
        al = -self._net(self.C, "q1.", f, p, self.actor(self.A, f, p)).mean()
        self.aopt.zero_grad()
        al.backward()
        self.aopt.step()
        self._polyak()
        return float(al.detach())
