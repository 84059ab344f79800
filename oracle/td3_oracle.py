"""CPU ORACLE for the TD3 hot path -- TEST INFRASTRUCTURE ONLY.

This module is a from-scratch numpy (float32) restatement of the reference's
``ReplayBuffer.sample`` + ``TD3.train`` gradient step.  It is the *checker*:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``td3_amd``) never
imports, links or executes anything under ``oracle/``.

Parity pin: ``tests/test_oracle_golden.py`` checks this restatement against
golden vectors produced by running the reference itself on CPU
(``tests/golden/make_golden.py``).

Reference functions restated here (``/root/reference/...``):

* ``my_replay_buffer.py:109-117``  ReplayBuffer_featured.add  -> ``FeaturedBuffer.add``
* ``my_replay_buffer.py:119-128``  ReplayBuffer_featured.sample (indices injected) -> ``FeaturedBuffer.gather``
* ``my_replay_buffer.py:46-69``    ReplayBuffer_particles.add/sample -> ``ParticleBuffer``
* ``TD3_featured.py:39-48``        Actor.forward  -> ``mlp_forward`` (+ tanh * max_action)
* ``TD3_featured.py:73-81``        Q.forward      -> ``mlp_forward`` on cat([s, a])
* ``TD3_featured.py:123-171``      TD3.train      -> ``featured_train_step``
* ``TD3_particles.py:52-69,103-119`` encoder + MLP -> ``encoder_forward`` / ``particle_*``
* ``TD3_particles.py:167-224``     TD3.train / _actor_learn -> ``particle_train_step``
* torch 2.10 ``_single_tensor_adam`` (torch/optim/adam.py:347, math :457-547) -> ``adam_``
* ``TD3_featured.py:33-35, 68-70`` norm="weight_normalization": torch ``weight_norm`` (dim 0)
  on every Linear, W = v * (g / ||v||) per output row, dg = (dW . v)/||v||,
  dv = (g/||v||) dW - (g (dW . v)/||v||^3) v  -> ``wn_weight`` / ``wn_grads``
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
LN_EPS = f32(1e-5)


# --------------------------------------------------------------------------- params
def wn_weight(g, v):
    """torch ``_weight_norm_interface`` (dim 0): W = v * (g / ||v||), ||v|| per output row."""
    n = np.sqrt((v.astype(np.float64) ** 2).sum(axis=1, keepdims=True)).astype(f32)
    return (v * (g / n)).astype(f32)


def wn_grads(gW, g, v):
    """Backward of ``wn_weight``: (dL/dg [N,1], dL/dv [N,K]) from dL/dW."""
    n = np.sqrt((v.astype(np.float64) ** 2).sum(axis=1, keepdims=True)).astype(f32)
    s = (gW.astype(np.float64) * v).sum(axis=1, keepdims=True).astype(f32)
    a = (g / n).astype(f32)
    b = (a * s / (n * n)).astype(f32)
    return (s / n).astype(f32), (a * gW - b * v).astype(f32)


def split_mlp(P, prefix, n_layers, norm, first_norm=False):
    """Collect (W, b) per Linear and (gamma, beta) per LayerNorm from a state dict."""
    if norm == "weight_normalization":
        lin = [(wn_weight(P[f"{prefix}linears.{i}.weight_g"], P[f"{prefix}linears.{i}.weight_v"]),
                P[f"{prefix}linears.{i}.bias"]) for i in range(n_layers)]
        return lin, None, None
    lin = [(P[f"{prefix}linears.{i}.weight"], P[f"{prefix}linears.{i}.bias"]) for i in range(n_layers)]
    ln = None
    ln0 = None
    if norm == "layer":
        ln = [(P[f"{prefix}lnorms.{i}.weight"], P[f"{prefix}lnorms.{i}.bias"]) for i in range(n_layers - 1)]
        if first_norm:
            ln0 = (P[f"{prefix}lnorm1.weight"], P[f"{prefix}lnorm1.bias"])
    return lin, ln, ln0


# --------------------------------------------------------------------------- layers
def layernorm_fwd(h, gamma, beta):
    """torch LayerNorm (biased var, eps 1e-5):  y = (x*rstd + (-mean*rstd))*gamma + beta."""
    h = h.astype(f32)
    mean = h.mean(axis=1, dtype=np.float64).astype(f32)
    d = h - mean[:, None]
    var = (d.astype(np.float64) ** 2).mean(axis=1).astype(f32)
    rstd = (f32(1.0) / np.sqrt(np.maximum(var, f32(0)) + LN_EPS)).astype(f32)
    u = (h * rstd[:, None] + (-mean * rstd)[:, None]) * gamma[None, :] + beta[None, :]
    return u.astype(f32), mean, rstd


def layernorm_bwd(gu, h, mean, rstd, gamma):
    """d/dh of LayerNorm given dL/du;  returns (dh, dgamma, dbeta)."""
    xhat = ((h - mean[:, None]) * rstd[:, None]).astype(f32)
    dgamma = (gu * xhat).sum(axis=0, dtype=np.float64).astype(f32)
    dbeta = gu.sum(axis=0, dtype=np.float64).astype(f32)
    gx = (gu * gamma[None, :]).astype(f32)
    n = f32(h.shape[1])
    m1 = gx.mean(axis=1, dtype=np.float64).astype(f32)
    m2 = (gx * xhat).mean(axis=1, dtype=np.float64).astype(f32)
    dh = rstd[:, None] * (gx - m1[:, None] - xhat * m2[:, None])
    del n
    return dh.astype(f32), dgamma, dbeta


def mlp_forward(lin, ln, x):
    """Linear -> ReLU -> LayerNorm on every hidden layer, bare last Linear.

    TD3_featured.py:41-46 (Actor) and :75-80 (Q): LN comes AFTER ReLU.
    Returns the last pre-activation and a cache for the backward.
    """
    cache = {"u": [x.astype(f32)], "h": [], "stats": []}
    a = x.astype(f32)
    L = len(lin)
    for i, (W, b) in enumerate(lin):
        z = (a @ W.T + b[None, :]).astype(f32)
        if i == L - 1:
            return z, cache
        h = np.maximum(z, f32(0))
        cache["h"].append(h)
        if ln is not None:
            a, mean, rstd = layernorm_fwd(h, *ln[i])
            cache["stats"].append((mean, rstd))
        else:
            a = h
        cache["u"].append(a)
    raise AssertionError("unreachable")


def mlp_backward(lin, ln, cache, gz_last):
    """Backward of ``mlp_forward`` given dL/d(last pre-activation).

    Returns (grads in state-dict order pieces, dL/dx of the MLP input).  ``cache["mask"]`` (optional,
    one bool array per hidden layer) replaces the relu' masks h > 0: the GPU parity tests pass the
    GPU's own masks, since a pre-activation within fp32 rounding of zero may fall on either side.
    """
    L = len(lin)
    gW = [None] * L
    gb = [None] * L
    gg = [None] * (L - 1)
    gbeta = [None] * (L - 1)
    gz = gz_last.astype(f32)
    for i in range(L - 1, -1, -1):
        W, _ = lin[i]
        u_in = cache["u"][i]
        gW[i] = (gz.T @ u_in).astype(f32)
        gb[i] = gz.sum(axis=0, dtype=np.float64).astype(f32)
        gu = (gz @ W).astype(f32)
        if i == 0:
            return (gW, gb, gg, gbeta), gu
        h = cache["h"][i - 1]
        if ln is not None:
            mean, rstd = cache["stats"][i - 1]
            gh, gg[i - 1], gbeta[i - 1] = layernorm_bwd(gu, h, mean, rstd, ln[i - 1][0])
        else:
            gh = gu
        mask = cache["mask"][i - 1] if "mask" in cache else h > 0
        gz = np.where(mask, gh, f32(0)).astype(f32)
    raise AssertionError("unreachable")


def pack_mlp_grads(prefix, grads, norm, extra=None, P=None):
    """Gradients in state-dict order; weight_normalization maps dW to (weight_g, weight_v)
    through the parameters ``P`` the backward ran with."""
    gW, gb, gg, gbeta = grads
    out = {}
    for i in range(len(gW)):
        if norm == "weight_normalization":
            out[f"{prefix}linears.{i}.bias"] = gb[i]
            out[f"{prefix}linears.{i}.weight_g"], out[f"{prefix}linears.{i}.weight_v"] = wn_grads(
                gW[i], P[f"{prefix}linears.{i}.weight_g"], P[f"{prefix}linears.{i}.weight_v"])
            continue
        out[f"{prefix}linears.{i}.weight"] = gW[i]
        out[f"{prefix}linears.{i}.bias"] = gb[i]
    if extra:
        out.update(extra)
    if norm == "layer":
        for i in range(len(gg)):
            out[f"{prefix}lnorms.{i}.weight"] = gg[i]
            out[f"{prefix}lnorms.{i}.bias"] = gbeta[i]
    return out


# --------------------------------------------------------------------------- optimiser
def adam_(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch ``_single_tensor_adam`` (adam.py:457-547), amsgrad/wd off, in place.

    exp_avg.lerp_(grad, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
    denom = sqrt(v)/sqrt(bc2) + eps;  p.addcdiv_(m, denom, -lr/bc1).
    Python-double scalars are cast to float32 the way ATen's CPU kernels do.
    """
    w = f32(1 - beta1)
    m += w * (g - m)
    v *= f32(beta2)
    v += (f32(1 - beta2) * g) * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    denom = np.sqrt(v) / f32(bc2 ** 0.5) + f32(eps)
    p += (f32(-step_size) * m) / denom


def polyak_(target, p, tau):
    """TD3_featured.py:167-171: target = tau*p + (1-tau)*target (float32 scalars)."""
    target[...] = f32(tau) * p + f32(1 - tau) * target


# --------------------------------------------------------------------------- replay
class FeaturedBuffer:
    """ReplayBuffer_featured (my_replay_buffer.py:72-128) without the RNG draw."""

    def __init__(self, sd, ad, max_size):
        self.max_size, self.ptr, self.size = max_size, 0, 0
        self.state = np.zeros((max_size, sd))
        self.action = np.zeros((max_size, ad))
        self.next_state = np.zeros((max_size, sd))
        self.reward = np.zeros((max_size, 1))
        self.not_done = np.zeros((max_size, 1))

    def add(self, s, a, s2, r, done):                         # :109-117
        self.state[self.ptr] = s
        self.action[self.ptr] = a
        self.next_state[self.ptr] = s2
        self.reward[self.ptr] = r
        self.not_done[self.ptr] = 1.0 - done
        self.ptr = (self.ptr + 1) % self.max_size
        self.size = min(self.size + 1, self.max_size)

    def gather(self, ind):                                   # :123-127 (f64 -> f32)
        return tuple(x[ind].astype(f32) for x in
                     (self.state, self.action, self.next_state, self.reward, self.not_done))


class ParticleBuffer:
    """ReplayBuffer_particles (my_replay_buffer.py:6-69) without the RNG draw."""

    def __init__(self, F, N, D, A, max_size):
        self.max_size, self.ptr, self.size = max_size, 0, 0
        self.state_features = np.zeros((max_size, F))
        self.state_particles = np.zeros((max_size, N, D))
        self.action = np.zeros((max_size, A))
        self.next_state_features = np.zeros((max_size, F))
        self.next_state_particles = np.zeros((max_size, N, D))
        self.reward = np.zeros((max_size, 1))
        self.not_done = np.zeros((max_size, 1))

    def add(self, s, a, s2, r, done):                         # :46-56
        self.state_features[self.ptr] = s[0]
        self.state_particles[self.ptr] = s[1]
        self.action[self.ptr] = a
        self.next_state_features[self.ptr] = s2[0]
        self.next_state_particles[self.ptr] = s2[1]
        self.reward[self.ptr] = r
        self.not_done[self.ptr] = 1.0 - done
        self.ptr = (self.ptr + 1) % self.max_size
        self.size = min(self.size + 1, self.max_size)

    def gather(self, ind):                                   # :58-69
        return tuple(x[ind].astype(f32) for x in
                     (self.state_features, self.state_particles, self.action,
                      self.next_state_features, self.next_state_particles,
                      self.reward, self.not_done))


# --------------------------------------------------------------------------- learner state
class Learner:
    """Everything ``TD3.train`` mutates: 4 param dicts, 2 Adam states, counters."""

    def __init__(self, actor, critic, *, max_action=1.0, discount=0.99, tau=0.005,
                 policy_noise=0.2, noise_clip=0.5, policy_freq=2, lr=1e-4, norm="layer",
                 cdq=True):
        cp = lambda d: {k: np.array(v, dtype=f32, copy=True) for k, v in d.items()}  # noqa: E731
        self.actor, self.critic = cp(actor), cp(critic)
        self.actor_target, self.critic_target = cp(actor), cp(critic)
        self.actor_m = {k: np.zeros_like(v) for k, v in self.actor.items()}
        self.actor_v = {k: np.zeros_like(v) for k, v in self.actor.items()}
        self.critic_m = {k: np.zeros_like(v) for k, v in self.critic.items()}
        self.critic_v = {k: np.zeros_like(v) for k, v in self.critic.items()}
        self.actor_step = 0
        self.critic_step = 0
        self.total_it = 0
        self.max_action, self.discount, self.tau = max_action, discount, tau
        self.policy_noise, self.noise_clip, self.policy_freq = policy_noise, noise_clip, policy_freq
        self.lr, self.norm, self.cdq = lr, norm, cdq

    def adam_critic(self, grads):
        self.critic_step += 1
        for k in self.critic:
            adam_(self.critic[k], grads[k], self.critic_m[k], self.critic_v[k], self.critic_step, self.lr)

    def adam_actor(self, grads):
        self.actor_step += 1
        for k in self.actor:
            adam_(self.actor[k], grads[k], self.actor_m[k], self.actor_v[k], self.actor_step, self.lr)

    def polyak(self):
        for k in self.critic:                                   # TD3_featured.py:167-168
            polyak_(self.critic_target[k], self.critic[k], self.tau)
        for k in self.actor:                                    # :170-171
            polyak_(self.actor_target[k], self.actor[k], self.tau)


# --------------------------------------------------------------------------- featured path
def featured_actor(P, norm, max_action, s):
    lin, ln, _ = split_mlp(P, "", 4, norm)
    z, cache = mlp_forward(lin, ln, s)
    t = np.tanh(z).astype(f32)
    return (f32(max_action) * t).astype(f32), (lin, ln, cache, t)


def featured_q(P, q, norm, s, a):
    lin, ln, _ = split_mlp(P, f"{q}.", 4, norm)
    x = np.concatenate([s, a], axis=1).astype(f32)              # TD3_featured.py:74
    z, cache = mlp_forward(lin, ln, x)
    return z, (lin, ln, cache)


def featured_train_step(L: Learner, batch, noise, record=None, grad_hook=None, masks=None):
    """One ``TD3_featured.TD3.train`` call (TD3_featured.py:123-171) on a gathered batch.

    ``batch`` = (state, action, next_state, reward, not_done) float32, ``noise`` =
    the N(0,1) draw of ``torch.randn_like(action)`` (:132).  ``grad_hook`` (data-parallel
    restatement) maps each phase's gradient dict before its Adam step, e.g. an
    all-reduce mean over ranks that each hold one shard of the global batch.  ``masks`` (tests):
    relu' masks per network ("q1", "q2", "actor", "aq": lists of 3 bool arrays) for the backward.
    """
    masks = masks or {}
    hook = grad_hook if grad_hook is not None else (lambda g: g)
    rec = record if record is not None else {}
    s, a, s2, r, nd = batch
    B = s.shape[0]
    L.total_it += 1                                                            # :124
    eps = np.clip(noise.astype(f32) * f32(L.policy_noise), -f32(L.noise_clip), f32(L.noise_clip))
    ta, _ = featured_actor(L.actor_target, L.norm, L.max_action, s2)
    next_a = np.clip(ta + eps, -f32(L.max_action), f32(L.max_action)).astype(f32)  # :135-137
    tq1, _ = featured_q(L.critic_target, "q1", L.norm, s2, next_a)
    tq2, _ = featured_q(L.critic_target, "q2", L.norm, s2, next_a)
    tq = np.minimum(tq1, tq2)                                                  # :141
    y = (r + (nd * f32(L.discount)) * tq).astype(f32)                        # :142
    q1, c1 = featured_q(L.critic, "q1", L.norm, s, a)                        # :145
    q2, c2 = featured_q(L.critic, "q2", L.norm, s, a)
    l1 = float(np.mean((q1 - y).astype(np.float64) ** 2))
    l2 = float(np.mean((q2 - y).astype(np.float64) ** 2))
    rec.update(ta_out=ta, next_action=next_a, y=y, q1=q1, q2=q2, critic_loss=l1 + l2,
               critic_loss_parts=(l1, l2))
    grads = {}
    for q, qv, (lin, ln, cache) in (("q1", q1, c1), ("q2", q2, c2)):
        if q in masks:
            cache["mask"] = masks[q]
        gq = (f32(2.0 / (B)) * (qv - y)).astype(f32)                          # d mse / dQ
        g, _ = mlp_backward(lin, ln, cache, gq)
        grads.update(pack_mlp_grads(f"{q}.", g, L.norm, P=L.critic))
    rec["critic_grads"] = grads
    L.adam_critic(hook(grads))                                                 # :151-153
    if L.total_it % L.policy_freq == 0:                                        # :156
        agrads = featured_actor_grads(L, s, rec, masks)
        L.adam_actor(hook(agrads))                                             # :162-164
        L.polyak()                                                             # :167-171
    return rec


def featured_actor_grads(L: Learner, s, record=None, masks=None):
    """The actor loss ``-Q1(s, pi(s)).mean()`` and its gradient over the actor's parameters
    (TD3_featured.py:159-161), with the critic as ``L.critic`` holds it (after the critic step)."""
    rec = record if record is not None else {}
    B = s.shape[0]
    masks = masks or {}
    pi, (alin, aln, acache, t) = featured_actor(L.actor, L.norm, L.max_action, s)
    aq1, (qlin, qln, qcache) = featured_q(L.critic, "q1", L.norm, s, pi)       # :159
    if "actor" in masks:
        acache["mask"] = masks["actor"]
    if "aq" in masks:
        qcache["mask"] = masks["aq"]
    rec.update(pi=pi, actor_q1=aq1, actor_loss=-float(np.mean(aq1, dtype=np.float64)))
    gq = np.full((B, 1), -1.0 / B, dtype=f32)
    _, gx = mlp_backward(qlin, qln, qcache, gq)
    gpi = gx[:, s.shape[1]:]
    gz = (gpi * f32(L.max_action)) * (f32(1) - t * t)                           # tanh'
    ag, _ = mlp_backward(alin, aln, acache, gz.astype(f32))
    agrads = pack_mlp_grads("", ag, L.norm, P=L.actor)
    rec["actor_grads"] = agrads
    return agrads


# --------------------------------------------------------------------------- particle path
def encoder_forward(P, prefix, part):
    """conv1 (1xD) -> ReLU -> conv2 (1x1) -> ReLU -> mean over N -> ReLU.

    TD3_particles.py:52-58 (Actor) / :104-109 (Q_network).
    part: [B, N, D] -> pooled [B, 128]
    """
    W1 = P[f"{prefix}conv1.weight"].reshape(P[f"{prefix}conv1.weight"].shape[0], -1)  # [256, D]
    b1 = P[f"{prefix}conv1.bias"]
    W2 = P[f"{prefix}conv2.weight"][:, :, 0]                                  # [128, 256]
    b2 = P[f"{prefix}conv2.bias"]
    Bn, N, D = part.shape
    x = part.reshape(Bn * N, D).astype(f32)
    h1 = np.maximum(x @ W1.T + b1[None, :], f32(0)).astype(f32)
    h2 = np.maximum(h1 @ W2.T + b2[None, :], f32(0)).astype(f32)
    pooled = h2.reshape(Bn, N, -1).mean(axis=1, dtype=np.float64).astype(f32)
    out = np.maximum(pooled, f32(0))
    return out, (x, h1, h2, pooled, W1, W2, Bn, N)


def encoder_backward(cache, g_out):
    x, h1, h2, pooled, W1, W2, Bn, N = cache
    gp = np.where(pooled > 0, g_out, f32(0)).astype(f32)
    gh2 = np.repeat(gp[:, None, :] / f32(N), N, axis=1).reshape(Bn * N, -1).astype(f32)
    gz2 = np.where(h2 > 0, gh2, f32(0)).astype(f32)
    gW2 = (gz2.T @ h1).astype(f32)
    gb2 = gz2.sum(axis=0, dtype=np.float64).astype(f32)
    gh1 = (gz2 @ W2).astype(f32)
    gz1 = np.where(h1 > 0, gh1, f32(0)).astype(f32)
    gW1 = (gz1.T @ x).astype(f32)
    gb1 = gz1.sum(axis=0, dtype=np.float64).astype(f32)
    return gW1, gb1, gW2, gb2


def particle_net(P, prefix, norm, feat, part, action=None, actor=False):
    """Actor / Q_network forward (TD3_particles.py:52-69 / :103-119)."""
    pooled, ecache = encoder_forward(P, prefix, part)
    parts = [pooled, feat.astype(f32)] + ([action.astype(f32)] if action is not None else [])
    x = np.concatenate(parts, axis=1).astype(f32)                          # :59 / :110
    lin, ln, ln0 = split_mlp(P, prefix, 4, norm, first_norm=True)
    if ln0 is not None:
        u0, m0, r0 = layernorm_fwd(x, *ln0)                                # lnorm1, :60-61
    else:
        u0, m0, r0 = x, None, None
    z, cache = mlp_forward(lin, ln, u0)
    if actor:
        out = np.tanh(z).astype(f32)                                       # :68 (no max_action)
    else:
        out = z
    return out, (ecache, x, (m0, r0), ln0, lin, ln, cache, z, out)


def particle_net_backward(norm, prefix, c, g_out, actor=False, need_input_grad=False):
    ecache, x, (m0, r0), ln0, lin, ln, cache, z, out = c
    gz = g_out.astype(f32)
    if actor:
        gz = (gz * (f32(1) - out * out)).astype(f32)
    g, gu0 = mlp_backward(lin, ln, cache, gz)
    extra = {}
    if ln0 is not None:
        gx, dg0, db0 = layernorm_bwd(gu0, x, m0, r0, ln0[0])
        extra = {f"{prefix}lnorm1.weight": dg0, f"{prefix}lnorm1.bias": db0}
    else:
        gx = gu0
    gpooled = gx[:, :128]
    gW1, gb1, gW2, gb2 = encoder_backward(ecache, gpooled)
    grads = {f"{prefix}conv1.weight": gW1.reshape(gW1.shape[0], 1, 1, -1),
             f"{prefix}conv1.bias": gb1,
             f"{prefix}conv2.weight": gW2[:, :, None],
             f"{prefix}conv2.bias": gb2}
    grads.update(pack_mlp_grads(prefix, g, norm, extra))
    return grads, gx


def _ordered(grads, P):
    return {k: grads[k] for k in P}


def particle_train_step(L: Learner, batch, noise, record=None):
    """One ``TD3_particles.TD3.train`` call (TD3_particles.py:167-224)."""
    rec = record if record is not None else {}
    f, p, a, f2, p2, r, nd = batch
    B = f.shape[0]
    L.total_it += 1
    eps = np.clip(noise.astype(f32) * f32(L.policy_noise), -f32(L.noise_clip), f32(L.noise_clip))
    ta, _ = particle_net(L.actor_target, "", L.norm, f2, p2, actor=True)
    next_a = (ta + eps).astype(f32)                                         # :179-181, no clamp
    qs = ("q1", "q2") if L.cdq else ("q1",)
    tqs = [particle_net(L.critic_target, f"{q}.", L.norm, f2, p2, next_a)[0] for q in qs]
    tq = np.minimum(tqs[0], tqs[1]) if L.cdq else tqs[0]
    y = (r + (nd * f32(L.discount)) * tq).astype(f32)                      # [B, A] broadcast
    grads = {}
    cur = []
    for q in qs:
        qv, c = particle_net(L.critic, f"{q}.", L.norm, f, p, a)
        cur.append(qv)
        gq = (f32(2.0 / qv.size) * (qv - y)).astype(f32)
        g, _ = particle_net_backward(L.norm, f"{q}.", c, gq)
        grads.update(g)
    losses = [float(np.mean((qv - y).astype(np.float64) ** 2)) for qv in cur]
    rec.update(ta_out=ta, next_action=next_a, y=y, critic_loss=sum(losses))
    for j, qv in enumerate(cur):
        rec[f"q{j + 1}"] = qv
    grads = _ordered(grads, L.critic)
    rec["critic_grads"] = grads
    L.adam_critic(grads)
    if L.total_it % L.policy_freq == 0:                                     # :206-207
        particle_actor_learn(L, f, p, rec)
    return rec


def particle_actor_learn(L: Learner, f, p, record=None):
    """``TD3_particles.TD3._actor_learn(state_features, state_particles)`` (TD3_particles.py:209-224):
    actor loss -mean Q1(s, pi(s)), the actor's Adam step, then Polyak of critic and actor.  It is
    also called on its own (evaluate_model.py:39-49); ``total_it`` is not touched."""
    rec = record if record is not None else {}
    pi, ac = particle_net(L.actor, "", L.norm, f, p, actor=True)             # :211
    aq1, qc = particle_net(L.critic, "q1.", L.norm, f, p, pi)              # :212
    rec.update(pi=pi, actor_q1=aq1, actor_loss=-float(np.mean(aq1, dtype=np.float64)))
    gq = np.full(aq1.shape, -1.0 / aq1.size, dtype=f32)
    _, gx = particle_net_backward(L.norm, "q1.", qc, gq)
    Fd = f.shape[1]
    gpi = gx[:, 128 + Fd:]
    ag, _ = particle_net_backward(L.norm, "", ac, gpi, actor=True)
    ag = _ordered(ag, L.actor)
    rec["actor_grads"] = ag
    L.adam_actor(ag)                                                        # :215-217
    L.polyak()                                                              # :219-224
    return rec


def featured_select_action(P, norm, max_action, state):
    """TD3_featured.py:113-115 at B=1."""
    out, _ = featured_actor(P, norm, max_action, np.asarray(state, dtype=f32).reshape(1, -1))
    return out.reshape(-1)
