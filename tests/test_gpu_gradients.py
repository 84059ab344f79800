"""Direct gradient parity of the fused dW + Adam kernels, through both Adam moments.

The fused dW stages feed Adam and never write the gradient itself (include/td3.h), so the
gradient is read back through the optimizer state: from zero moments one Adam step leaves
exp_avg = 0.1 g and exp_avg_sq = 0.001 g^2 (torch ``_single_tensor_adam``, SURVEY.md §8 a8;
TD3_featured.py:151-153, 162-164).  Both are compared against the oracle at SURVEY §8c's
gradient tolerance: rtol 1e-4 of the tensor scale for exp_avg (2e-4 for exp_avg_sq, which
is quadratic in g).  Post-Adam parameters alone cannot show a gradient-scale error: at step 1
they are theta - lr*sign(g).

Cases: HalfCheetah B=256 (dw_kernel, Adam fused per tile), Humanoid B=128 and B=1024 (the
split-K dwsk_kernel + dwsk_combine_kernel path of B >= 512), particles (encoder dW slabs +
enc_adam_kernel).  The critic gradient is checked at step 1 and, teacher-forced, at step 2.  The
actor gradient (step 2, a policy step) reads the critic the step has just updated; the oracle's
actor gradient is therefore computed on the GPU's updated critic, so that the two critics'
2*lr sign-flip differences (§8c) do not enter the comparison.

ReLU masks: a pre-activation within fp32 rounding of zero may land on either side in two correct
fp32 implementations.  At Humanoid widths, B = 1024, the second step has Q2 layer-1 pre-activation
z[94, 396] = -9.6e-8.  The GPU's sum came out positive and the oracle's negative. That one relu'
flip moved q2.linears.1.weight by 1.7e-2 of its scale in row 396, and every layer below it by
~1e-3 (tools/grad_diag.py, round 4). Every GPU variant gave the same numbers: the dW kernels, the
sequential critic and the old 64x64 dW all agreed. So the featured cases read the GPU's own masks
(td3_debug_activation: the post-ReLU activations H of Q1, Q2, the actor and Q1(s, pi)), and the
oracle's backward uses them (oracle mlp_backward cache["mask"]).  Each tensor is also checked
against the oracle in float64 from the same state (same masks): within rtol of it, or no further
from it than 3x the fp32 oracle -- the reference's own fp32 noise floor.
"""
import contextlib

import numpy as np
import pytest

from helpers import featured_setup, featured_setup_dims, gen, orc, particle_setup
from test_gpu_parity import _load_oracle_state, _make as _make_featured, _rel_to_max
from test_gpu_particles import _make as _make_particles

pytestmark = pytest.mark.gpu

M_RTOL, V_RTOL = 1e-4, 2e-4

CASES = {
    "hc_layer": lambda: ("featured", featured_setup("hc_layer")),
    "hum_layer": lambda: ("featured", featured_setup("hum_layer")),
    "hum_b1024": lambda: ("featured", featured_setup_dims(376, 17, 0.4, "layer", B=1024)),
    "part_layer": lambda: ("particles", particle_setup("part_layer")),
}


def _moments(opt):
    st = opt.state_dict()["state"]
    return ([st[i]["exp_avg"].numpy() for i in range(len(st))],
            [st[i]["exp_avg_sq"].numpy() for i in range(len(st))],
            [float(st[i]["step"]) for i in range(len(st))])


class _Float64Oracle:
    """The oracle's arithmetic in float64 while inside (it types every array through orc.f32)."""

    def __enter__(self):
        self.saved = orc.f32
        orc.f32 = np.float64
        return self

    def __exit__(self, *exc):
        orc.f32 = self.saved
        return False


def _copy_learner(L, kw):
    """A float64 Learner in L's exact state (parameters, targets, moments, counters)."""
    with _Float64Oracle():
        L64 = orc.Learner(L.actor, L.critic, **kw)
        for name in ("actor_target", "critic_target", "actor_m", "actor_v", "critic_m", "critic_v"):
            setattr(L64, name, {k: np.asarray(v, np.float64).copy() for k, v in getattr(L, name).items()})
    L64.total_it, L64.critic_step, L64.actor_step = L.total_it, L.critic_step, L.actor_step
    return L64


def _check(opt, m32, v32, m64, v64, step, what):
    ms, vs, steps = _moments(opt)
    assert set(steps) == {float(step)}, (what, steps)
    assert len(ms) == len(m32)
    for i, k in enumerate(m32):
        assert ms[i].shape == m32[k].shape, (what, k)
        assert np.abs(m32[k]).max() > 0, (what, k, "zero reference gradient")
        for name, gpu, o32, o64, tol in (("exp_avg", ms[i], m32[k], m64[k], M_RTOL),
                                          ("exp_avg_sq", vs[i], v32[k], v64[k], V_RTOL)):
            e_gpu, e_o32 = _rel_to_max(gpu, o64), _rel_to_max(o32, o64)
            assert e_gpu <= max(tol, 3.0 * e_o32), (what, k, name, e_gpu, e_o32)


def _draw(rs, S, kind):
    B = S["B"]
    ad = S["A"] if kind == "particles" else S["ad"]
    return rs.randint(0, gen.BUFFER_ROWS, size=B), rs.standard_normal((B, ad)).astype(np.float32)


def _step64(L, kind, batch, noise, kw, masks=None):
    """The oracle step in float64 from L's state (L untouched)."""
    L64 = _copy_learner(L, kw)
    with _Float64Oracle():
        b64 = tuple(np.asarray(x, np.float64) for x in batch)
        if kind == "particles":
            orc.particle_train_step(L64, b64, np.asarray(noise, np.float64))
        else:
            orc.featured_train_step(L64, b64, np.asarray(noise, np.float64), masks=masks)
    return L64


def _gpu_masks(pol, B, actor_step):
    """The relu' masks of the GPU's last step (td3_debug_activation: H > 0) for every network the
    step backpropagates through: Q1, Q2 (s, a); on a policy step the actor (s) and Q1 (s, pi)."""
    import ctypes as C
    from td3_amd import _lib
    q, a = [500, 400, 200], [500, 400, 300]
    evals = [("q1", 1, q), ("q2", 2, q)] + ([("actor", 3, a), ("aq", 6, q)] if actor_step else [])
    out = {}
    for name, ev, widths in evals:
        ms = []
        for layer, n in enumerate(widths):
            buf = np.empty((B, n), np.float32)
            _lib.check(pol._lib.td3_debug_activation(pol._h, ev, layer, buf.ctypes.data_as(C.c_void_p), B, n),
                       "td3_debug_activation")
            ms.append(buf > 0)
        out[name] = ms
    return out


@pytest.mark.parametrize("case", list(CASES))
def test_gradients_through_adam_moments(case):
    kind, S = CASES[case]()
    make = _make_particles if kind == "particles" else _make_featured
    step_fn = orc.particle_train_step if kind == "particles" else orc.featured_train_step
    pol, rb = make(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(11)

    featured = kind != "particles"
    kw_step = (lambda m: {"masks": m}) if featured else (lambda m: {})

    # step 1 (critic only) from zero moments
    idx, noise = _draw(rs, S, kind)
    batch = S["buf"].gather(idx)
    pol.train_step(rb, S["B"], indices=idx, noise=noise)
    assert pol._counters() == (1, 1, 0)
    masks = _gpu_masks(pol, S["B"], False) if featured else None
    if featured:        # the GPU's masks differ from the oracle's only at |z| ~ 0
        om, near = _own_masks(L.critic, L.actor, S["norm"], S["ma"], batch[0], batch[1], False)
        _check_mask_flips(masks, om, near, (case, "step 1"))
    L64 = _step64(L, kind, batch, noise, S["kw"], masks)
    step_fn(L, batch, noise, **kw_step(masks))
    _check(pol.critic_optimizer, L.critic_m, L.critic_v, L64.critic_m, L64.critic_v, 1, (case, "critic step 1"))

    # step 2 (critic + actor), teacher-forced from the oracle's state after step 1
    _load_oracle_state(pol, L)
    actor0 = {k: v.copy() for k, v in L.actor.items()}
    idx, noise = _draw(rs, S, kind)
    batch = S["buf"].gather(idx)
    pol.train_step(rb, S["B"], indices=idx, noise=noise)
    assert pol._counters() == (2, 2, 1)
    masks = _gpu_masks(pol, S["B"], True) if featured else None
    if featured:
        om, near = _own_masks(L.critic, L.actor, S["norm"], S["ma"], batch[0], batch[1], False)
        _check_mask_flips({k: masks[k] for k in om}, om, near, (case, "step 2"))
    L64 = _step64(L, kind, batch, noise, S["kw"], masks)
    step_fn(L, batch, noise, **kw_step(masks))
    _check(pol.critic_optimizer, L.critic_m, L.critic_v, L64.critic_m, L64.critic_v, 2, (case, "critic step 2"))

    # the actor gradient on the critic this step produced on the GPU (fp32 and float64 oracles)
    crit = pol.critic.numpy_dict()
    Lc = orc.Learner(actor0, crit, **S["kw"])
    with _Float64Oracle():
        Lc64 = orc.Learner(actor0, crit, **S["kw"])
    for Lx, f64 in ((Lc, False), (Lc64, True)):
        ctx = _Float64Oracle() if f64 else contextlib.nullcontext()
        with ctx:
            if kind == "particles":
                orc.particle_actor_learn(Lx, *(np.asarray(x, np.float64 if f64 else np.float32) for x in batch[:2]))
            else:
                Lx.adam_actor(orc.featured_actor_grads(Lx, np.asarray(batch[0], np.float64 if f64 else np.float32),
                                                       masks=masks))
    _check(pol.actor_optimizer, Lc.actor_m, Lc.actor_v, Lc64.actor_m, Lc64.actor_v, 1, (case, "actor"))


# ------------------------------------------------------------------ Humanoid B = 1024 on the oracle's own masks
MASK_EPS = 1e-6          # |z| below this fraction of a layer's max |z| is "within fp32 rounding of 0"


def _preacts64(P, prefix, norm, x):
    """float64 pre-activations z of the hidden layers of one MLP (TD3_featured.py:41-46 / :75-80)."""
    with _Float64Oracle():
        lin, ln, _ = orc.split_mlp(P, prefix, 4, norm)
        lin = [(np.asarray(W, np.float64), np.asarray(b, np.float64)) for W, b in lin]
        _, cache = orc.mlp_forward(lin, ln, np.asarray(x, np.float64))
    return [cache["u"][i] @ lin[i][0].T + lin[i][1][None, :] for i in range(3)]


def _own_masks(crit, actor, norm, ma, s, a, with_actor):
    """The oracle's own relu' masks (z > 0 in float64) and each layer's near-zero set."""
    nets = {"q1": _preacts64(crit, "q1.", norm, np.concatenate([s, a], 1)),
            "q2": _preacts64(crit, "q2.", norm, np.concatenate([s, a], 1))}
    if with_actor:
        nets["actor"] = _preacts64(actor, "", norm, s)
        with _Float64Oracle():
            pi, _ = orc.featured_actor({k: np.asarray(v, np.float64) for k, v in actor.items()}, norm, ma,
                                       np.asarray(s, np.float64))
        nets["aq"] = _preacts64(crit, "q1.", norm, np.concatenate([s, pi], 1))
    masks = {k: [z > 0 for z in zs] for k, zs in nets.items()}
    near = {k: [np.abs(z) < MASK_EPS * np.abs(z).max() for z in zs] for k, zs in nets.items()}
    return masks, near


def _check_mask_flips(gm, om, near, what):
    """the GPU's masks may differ from the oracle's only at pre-activations within fp32
    rounding of zero, at most as many as there are such pre-activations."""
    flips = 0
    for k in om:
        for layer, (g, o, nz) in enumerate(zip(gm[k], om[k], near[k])):
            bad = g != o
            assert not (bad & ~nz).any(), (what, k, layer, int((bad & ~nz).sum()), "flip off the near-zero set")
            assert bad.sum() <= nz.sum(), (what, k, layer)
            flips += int(bad.sum())
    return flips


def _check_own(opt, own64, gm64, step, what):
    """exp_avg / exp_avg_sq against the float64 oracle on its OWN masks: within rtol of the tensor
    scale, plus (element by element) the effect of the flipped relu' decisions -- the float64
    difference between the oracle on the GPU's masks and on its own.  Elements the flips do not
    reach get the plain rtol check."""
    ms, vs, steps = _moments(opt)
    assert set(steps) == {float(step)}, (what, steps)
    for i, k in enumerate(own64[0]):
        for name, gpu, o64, f64, tol in (("exp_avg", ms[i], own64[0][k], gm64[0][k], M_RTOL),
                                          ("exp_avg_sq", vs[i], own64[1][k], gm64[1][k], V_RTOL)):
            o64, f64 = np.asarray(o64, np.float64), np.asarray(f64, np.float64)
            allow = tol * np.abs(o64).max() + 1.01 * np.abs(f64 - o64)
            err = np.abs(np.asarray(gpu, np.float64) - o64)
            assert (err <= allow).all(), (what, k, name, float((err - allow).max()), float(np.abs(o64).max()))


def test_humanoid_b1024_gradients_on_oracle_masks():
    """VERDICT r04 weak #1c: the Humanoid B = 1024 gradient (split-K dW) on the oracle's own masks."""
    S = featured_setup_dims(376, 17, 0.4, "layer", B=1024)
    pol, rb = _make_featured(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(11)
    total_flips = 0
    for step in (1, 2):
        if step == 2:
            _load_oracle_state(pol, L)
        actor0 = {k: v.copy() for k, v in L.actor.items()}
        idx, noise = _draw(rs, S, "featured")
        batch = S["buf"].gather(idx)
        pol.train_step(rb, S["B"], indices=idx, noise=noise)
        actor_step = step == 2
        gm = _gpu_masks(pol, S["B"], actor_step)
        om, near = _own_masks(L.critic, L.actor, "layer", S["ma"], batch[0], batch[1], False)
        total_flips += _check_mask_flips({k: gm[k] for k in om}, om, near, ("critic", step))
        own = _step64(L, "featured", batch, noise, S["kw"])
        flip = _step64(L, "featured", batch, noise, S["kw"], gm)
        _check_own(pol.critic_optimizer, (own.critic_m, own.critic_v), (flip.critic_m, flip.critic_v), step,
                   ("critic", step))
        orc.featured_train_step(L, batch, noise)
    # the actor gradient (step 2) through the critic the GPU produced, on the oracle's own masks
    crit = pol.critic.numpy_dict()
    om, near = _own_masks(crit, actor0, "layer", S["ma"], batch[0], batch[1], True)
    total_flips += _check_mask_flips({k: gm[k] for k in ("actor", "aq")}, {k: om[k] for k in ("actor", "aq")},
                                     near, "actor")
    res = []
    for masks in (None, {k: gm[k] for k in ("actor", "aq")}):
        with _Float64Oracle():
            Lx = orc.Learner(actor0, crit, **S["kw"])
            Lx.adam_actor(orc.featured_actor_grads(Lx, np.asarray(batch[0], np.float64), masks=masks))
        res.append((Lx.actor_m, Lx.actor_v))
    _check_own(pol.actor_optimizer, res[0], res[1], 1, "actor")
    print(f"relu' decisions that differ from the oracle's (all at |z| < {MASK_EPS} of scale): {total_flips}")
