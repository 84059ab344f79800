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
"""
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


def _check(opt, m_ref, v_ref, step, what):
    ms, vs, steps = _moments(opt)
    assert set(steps) == {float(step)}, (what, steps)
    assert len(ms) == len(m_ref)
    for i, k in enumerate(m_ref):
        assert ms[i].shape == m_ref[k].shape, (what, k)
        assert np.abs(m_ref[k]).max() > 0, (what, k, "zero reference gradient")
        em, ev = _rel_to_max(ms[i], m_ref[k]), _rel_to_max(vs[i], v_ref[k])
        assert em <= M_RTOL, (what, k, "exp_avg", em)
        assert ev <= V_RTOL, (what, k, "exp_avg_sq", ev)


def _draw(rs, S, kind):
    B = S["B"]
    ad = S["A"] if kind == "particles" else S["ad"]
    return rs.randint(0, gen.BUFFER_ROWS, size=B), rs.standard_normal((B, ad)).astype(np.float32)


@pytest.mark.parametrize("case", list(CASES))
def test_gradients_through_adam_moments(case):
    kind, S = CASES[case]()
    make = _make_particles if kind == "particles" else _make_featured
    step_fn = orc.particle_train_step if kind == "particles" else orc.featured_train_step
    pol, rb = make(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(11)

    # step 1 (critic only) from zero moments
    idx, noise = _draw(rs, S, kind)
    step_fn(L, S["buf"].gather(idx), noise)
    pol.train_step(rb, S["B"], indices=idx, noise=noise)
    assert pol._counters() == (1, 1, 0)
    _check(pol.critic_optimizer, L.critic_m, L.critic_v, 1, (case, "critic step 1"))

    # step 2 (critic + actor), teacher-forced from the oracle's state after step 1
    _load_oracle_state(pol, L)
    actor0 = {k: v.copy() for k, v in L.actor.items()}
    idx, noise = _draw(rs, S, kind)
    batch = S["buf"].gather(idx)
    step_fn(L, batch, noise)
    pol.train_step(rb, S["B"], indices=idx, noise=noise)
    assert pol._counters() == (2, 2, 1)
    _check(pol.critic_optimizer, L.critic_m, L.critic_v, 2, (case, "critic step 2"))

    # the actor gradient on the critic this step produced on the GPU
    Lc = orc.Learner(actor0, pol.critic.numpy_dict(), **S["kw"])
    if kind == "particles":
        orc.particle_actor_learn(Lc, batch[0], batch[1])
    else:
        Lc.adam_actor(orc.featured_actor_grads(Lc, batch[0]))
    _check(pol.actor_optimizer, Lc.actor_m, Lc.actor_v, 1, (case, "actor"))
