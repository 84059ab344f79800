"""Pin the CPU oracle against golden vectors produced by the reference itself.

The goldens (tests/golden/*.npz) come from running /root/reference's
TD3_featured.TD3.train / TD3_particles.TD3.train on CPU with recorded RNG draws
(tests/golden/make_golden.py).  Every step is replayed free-running from the same
initial state with the recorded indices and noise.
"""
import numpy as np
import pytest

from helpers import gen, orc, load_golden, featured_setup, particle_setup


def _rel_to_max(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / (np.abs(b).max() + 1e-30))


def _check_groups(Lr, G, p, param_atol):
    for grp, P, sb in (("actor", Lr.actor, 0), ("critic", Lr.critic, 500),
                       ("actor_target", Lr.actor_target, 0),
                       ("critic_target", Lr.critic_target, 500)):
        for i, (k, v) in enumerate(P.items()):
            st, smp = gen.summarize(v, salt=sb + i)
            ref = G[f"{p}/{grp}/{k}/samples"]
            assert np.abs(smp - ref).max() <= param_atol, (p, grp, k)
            np.testing.assert_allclose(st[0], G[f"{p}/{grp}/{k}/stats"][0],
                                       atol=1e-3 * max(1.0, np.sqrt(v.size) * 1e-3))
    for grp, M, V, sb in (("critic_opt", Lr.critic_m, Lr.critic_v, 500),
                          ("actor_opt", Lr.actor_m, Lr.actor_v, 0)):
        if f"{p}/{grp}/step" not in G:
            continue
        for i, k in enumerate(M):
            for key, arr in (("exp_avg", M[k]), ("exp_avg_sq", V[k])):
                st, smp = gen.summarize(arr, salt=sb + i)
                ref = G[f"{p}/{grp}/{key}/{k}/samples"]
                scale = np.abs(ref).max() + 1e-30
                assert np.abs(smp - ref).max() <= 1e-3 * scale, (p, grp, key, k)


def _check_grads(rec, G, p):
    if "actor_grads" in rec:
        grads, grp, sb = rec["actor_grads"], "actor", 0
    else:
        grads, grp, sb = rec["critic_grads"], "critic", 500
    for i, (k, v) in enumerate(grads.items()):
        st, smp = gen.summarize(v, salt=sb + i)
        ref = G[f"{p}/grad/{grp}/{k}/samples"]
        assert _rel_to_max(smp, ref) <= 2e-4, (p, grp, k, _rel_to_max(smp, ref))


@pytest.mark.parametrize("name", list(gen.FEATURED_CONFIGS))
def test_featured_oracle_matches_reference(name):
    G = load_golden("featured", name)
    S = featured_setup(name)
    np.testing.assert_allclose(
        G["buffer/checksum"],
        [S["buf"].state.sum(), S["buf"].action.sum(), S["buf"].next_state.sum(),
         S["buf"].reward.sum(), S["buf"].not_done.sum()], rtol=1e-12)
    Lr = orc.Learner(S["actor"], S["critic"], **S["kw"])
    for step in range(1, S["steps"] + 1):
        p = f"step{step}"
        idx = G[f"{p}/idx"]
        assert idx.shape == (S["B"],) and idx.min() >= 0 and idx.max() < gen.BUFFER_ROWS
        rec = orc.featured_train_step(Lr, S["buf"].gather(idx), G[f"{p}/noise"])
        for k in ("y", "q1", "q2", "ta_out"):
            assert _rel_to_max(rec[k], G[f"{p}/{k}"]) <= 2e-5, (p, k)
        np.testing.assert_allclose(rec["critic_loss"], G[f"{p}/critic_loss"], rtol=1e-5)
        assert bool(G[f"{p}/actor_step"]) == ("actor_loss" in rec)
        if "actor_loss" in rec:
            np.testing.assert_allclose(rec["actor_loss"], G[f"{p}/actor_loss"], rtol=1e-5)
            assert _rel_to_max(rec["pi"], G[f"{p}/pi"]) <= 2e-5
        _check_grads(rec, G, p)
        _check_groups(Lr, G, p, param_atol=2e-5)


@pytest.mark.parametrize("name", list(gen.PARTICLE_CONFIGS))
def test_particle_oracle_matches_reference(name):
    G = load_golden("particles", name)
    S = particle_setup(name)
    Lr = orc.Learner(S["actor"], S["critic"], **S["kw"])
    for step in range(1, S["steps"] + 1):
        p = f"step{step}"
        rec = orc.particle_train_step(Lr, S["buf"].gather(G[f"{p}/idx"]), G[f"{p}/noise"])
        for k in ("y", "q1", "ta_out"):
            assert _rel_to_max(rec[k], G[f"{p}/{k}"]) <= 2e-5, (p, k)
        np.testing.assert_allclose(rec["critic_loss"], G[f"{p}/critic_loss"], rtol=1e-5)
        if "actor_loss" in rec:
            np.testing.assert_allclose(rec["actor_loss"], G[f"{p}/actor_loss"], rtol=1e-5)
        _check_grads(rec, G, p)
        _check_groups(Lr, G, p, param_atol=5e-5)


def test_buffer_ring_semantics():
    """my_replay_buffer.py:109-117: ptr wraps, size saturates, not_done = 1 - done."""
    b = orc.FeaturedBuffer(2, 1, 3)
    for i in range(5):
        b.add([i, i], [i], [i + 1, i + 1], float(i), float(i % 2))
    assert b.ptr == 2 and b.size == 3
    np.testing.assert_array_equal(b.state[:, 0], [3, 4, 2])
    np.testing.assert_array_equal(b.not_done[:, 0], [0, 1, 1])
