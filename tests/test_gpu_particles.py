"""GPU parity of the TD3_particles path (encoder kernels + particle heads) against the oracle.

Same tolerances as tests/test_gpu_parity.py.  The golden fixtures hold
F=7, N=16, D=9, A=3, B=32 (one particle tile); ``test_many_particle_tiles`` runs N=350
(11 tiles, the last one masked) against the oracle directly.
"""
import numpy as np
import pytest

from helpers import gen, orc, load_golden, particle_setup
from test_gpu_parity import _load_oracle_state, _params_close, _rel_to_max

pytestmark = pytest.mark.gpu


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def _make(S, use_graph=True, rows=gen.BUFFER_ROWS, data=None):
    from td3_amd.TD3_particles import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_particles
    F, N, D, A = S["F"], S["N"], S["D"], S["A"]
    obs = (Box((F,)), Box((N, D)))
    pol = TD3(obs, Box((A,)), norm=S["norm"], CDQ=S["cdq"], use_graph=use_graph, init="none")
    pol.set_weights(S["actor"], S["critic"])
    rb = ReplayBuffer_particles(obs, Box((A,)), max_size=rows)
    f, p, a, f2, p2, r, d = data if data is not None else gen.fill_particle_buffer(F, N, D, A, rows, gen.SEED)
    rb.add_batch(f, p, a, f2, p2, r, d)
    return pol, rb


def _check_step(out, rec, pol, L, what):
    assert _rel_to_max(out["y"], rec["y"]) <= 1e-5, (what, "y")
    assert _rel_to_max(out["q1"], rec["q1"]) <= 1e-5, (what, "q1")
    if "q2" in rec:
        assert _rel_to_max(out["q2"], rec["q2"]) <= 1e-5, (what, "q2")
    np.testing.assert_allclose(out["critic_loss"], rec["critic_loss"], rtol=1e-5)
    assert out["actor_step"] == ("actor_loss" in rec)
    if out["actor_step"]:
        np.testing.assert_allclose(out["actor_loss"], rec["actor_loss"], rtol=1e-5, atol=1e-7)
    _params_close(pol.critic.numpy_dict(), L.critic, L.lr, (what, "critic"))
    _params_close(pol.critic_target.numpy_dict(), L.critic_target, L.lr, (what, "critic_target"))
    _params_close(pol.actor.numpy_dict(), L.actor, L.lr, (what, "actor"))
    _params_close(pol.actor_target.numpy_dict(), L.actor_target, L.lr, (what, "actor_target"))
    assert pol._counters() == (L.total_it, L.critic_step, L.actor_step)


def test_particle_sample_bit_exact():
    S = particle_setup("part_layer")
    pol, rb = _make(S)
    idx = np.random.RandomState(5).randint(0, gen.BUFFER_ROWS, size=40)
    out = rb.sample(40, indices=idx)
    ref = S["buf"].gather(idx)
    for o, r in zip(out, ref):
        np.testing.assert_array_equal(o.cpu().numpy().reshape(r.shape), r)


@pytest.mark.parametrize("name", list(gen.PARTICLE_CONFIGS))
def test_particle_step_teacher_forced(name):
    G = load_golden("particles", name)
    S = particle_setup(name)
    pol, rb = _make(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    for step in range(1, S["steps"] + 1):
        p = f"step{step}"
        idx, noise = G[f"{p}/idx"], G[f"{p}/noise"]
        _load_oracle_state(pol, L)
        rec = orc.particle_train_step(L, S["buf"].gather(idx), noise)
        out = pol.train_step(rb, S["B"], indices=idx, noise=noise, stats=True)
        np.testing.assert_array_equal(out["idx"], idx)
        _check_step(out, rec, pol, L, p)
        assert _rel_to_max(out["y"], G[f"{p}/y"]) <= 2e-5


@pytest.mark.parametrize("name", list(gen.PARTICLE_CONFIGS))
def test_particle_free_running_matches_golden(name):
    """Both steps free-running from the reference's initial state, against its goldens."""
    G = load_golden("particles", name)
    S = particle_setup(name)
    pol, rb = _make(S)
    for step in range(1, S["steps"] + 1):
        p = f"step{step}"
        out = pol.train_step(rb, S["B"], indices=G[f"{p}/idx"], noise=G[f"{p}/noise"], stats=True)
        assert _rel_to_max(out["y"], G[f"{p}/y"]) <= 5e-5
        assert _rel_to_max(out["q1"], G[f"{p}/q1"]) <= 5e-5
        np.testing.assert_allclose(out["critic_loss"], float(G[f"{p}/critic_loss"]), rtol=5e-5)
        for grp, view, sb in (("actor", pol.actor, 0), ("critic", pol.critic, 500),
                              ("critic_target", pol.critic_target, 500)):
            for i, (k, v) in enumerate(view.numpy_dict().items()):
                key = f"{p}/{grp}/{k}/samples"
                if key not in G:
                    continue
                _, smp = gen.summarize(v, salt=sb + i)
                assert np.abs(smp - G[key]).max() <= 2.5e-4, (p, grp, k)


def test_particle_graph_equals_eager():
    S = particle_setup("part_layer")
    G = load_golden("particles", "part_layer")
    outs = []
    for use_graph in (False, True):
        pol, rb = _make(S, use_graph=use_graph)
        for step in range(1, 3):
            p = f"step{step}"
            pol.train_step(rb, S["B"], indices=G[f"{p}/idx"], noise=G[f"{p}/noise"])
        outs.append((pol.actor.flat(), pol.critic.flat(), pol.critic_target.flat()))
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_particle_philox_path():
    """Production path: Philox rows / noise read back and replayed through the oracle."""
    S = particle_setup("part_layer")
    pol, rb = _make(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    for step in range(1, 3):
        _load_oracle_state(pol, L)
        out = pol.train_step(rb, S["B"], stats=True)
        assert out["idx"].min() >= 0 and out["idx"].max() < gen.BUFFER_ROWS
        rec = orc.particle_train_step(L, S["buf"].gather(out["idx"]), out["noise"])
        _check_step(out, rec, pol, L, step)


def test_particle_select_action_and_eval_q():
    S = particle_setup("part_layer")
    pol, _ = _make(S)
    rs = np.random.RandomState(1)
    for _ in range(2):
        f = rs.standard_normal(S["F"]).astype(np.float32)
        p = rs.standard_normal((S["N"], S["D"])).astype(np.float32)
        a = pol.select_action((f, p))
        ref, _ = orc.particle_net(S["actor"], "", S["norm"], f[None], p[None], actor=True)
        np.testing.assert_allclose(a, ref[0], rtol=1e-5, atol=1e-6)
        q = pol.eval_q((f, p), a)
        for j, qn in enumerate(("q1", "q2")):
            qr, _ = orc.particle_net(S["critic"], f"{qn}.", S["norm"], f[None], p[None], a[None])
            np.testing.assert_allclose(q[j], qr[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n", [3, 40])
def test_particle_select_action_batch(n):
    """Several particle queries in one call (mapped host I/O up to 256 padded rows)."""
    from td3_amd import _lib
    S = particle_setup("part_layer")
    pol, _ = _make(S)
    rs = np.random.RandomState(n)
    f = rs.standard_normal((n, S["F"])).astype(np.float32)
    p = rs.standard_normal((n, S["N"], S["D"])).astype(np.float32)
    out = np.empty((n, S["A"]), np.float32)
    _lib.check(pol._lib.td3_select_action_particles(pol._h, _lib.fptr(f), _lib.fptr(p), _lib.fptr(out), n),
               "td3_select_action_particles")
    ref, _ = orc.particle_net(S["actor"], "", S["norm"], f, p, actor=True)
    assert float(np.abs(out - ref).max()) <= 1e-5 * float(np.abs(ref).max()) + 1e-6


def test_particle_foreign_buffer_path():
    S = particle_setup("part_nocdq")
    G = load_golden("particles", "part_nocdq")
    pol, _ = _make(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    idx, noise = G["step1/idx"], G["step1/noise"]

    class Foreign:
        def sample(self, B):
            import torch
            return tuple(torch.from_numpy(x) for x in S["buf"].gather(idx))

    rec = orc.particle_train_step(L, S["buf"].gather(idx), noise)
    out = pol.train_step(Foreign(), S["B"], noise=noise, stats=True)
    assert _rel_to_max(out["y"], rec["y"]) <= 1e-5
    _params_close(pol.critic.numpy_dict(), L.critic, 1e-4, "critic")


def test_many_particle_tiles():
    """N = 350 particles (11 tiles of 32, last one masked), two steps, against the oracle."""
    F, N, D, A, B, rows = 7, 350, 9, 3, 16, 64
    S = dict(F=F, N=N, D=D, A=A, norm="layer", cdq=True, B=B)
    S["actor"] = gen.init_params(gen.particle_actor_shapes(F, D, A, "layer"), 11)
    S["critic"] = gen.init_params(gen.particle_critic_shapes(F, D, A, "layer", True), 12)
    data = gen.fill_particle_buffer(F, N, D, A, rows, 13)
    pol, rb = _make(S, rows=rows, data=data)
    buf = orc.ParticleBuffer(F, N, D, A, rows)
    f, p, a, f2, p2, r, d = data
    for i in range(rows):
        buf.add((f[i], p[i]), a[i], (f2[i], p2[i]), r[i], d[i])
    L = orc.Learner(S["actor"], S["critic"], norm="layer", cdq=True)
    rs = np.random.RandomState(14)
    for step in range(1, 3):
        idx = rs.randint(0, rows, B)
        noise = rs.standard_normal((B, A)).astype(np.float32)
        _load_oracle_state(pol, L)
        rec = orc.particle_train_step(L, buf.gather(idx), noise)
        out = pol.train_step(rb, B, indices=idx, noise=noise, stats=True)
        _check_step(out, rec, pol, L, step)
