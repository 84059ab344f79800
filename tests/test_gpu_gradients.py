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
