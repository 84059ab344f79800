"""TD3_particles surface beyond train(): ``_actor_learn`` on its own and checkpoint interop.

* ``TD3._actor_learn(state_features, state_particles)`` (TD3_particles.py:209-224), which
  ``evaluate_model.py:39-49`` calls outside ``train``: the actor loss, the actor's Adam step and the
  Polyak update of critic and actor against ``oracle.particle_actor_learn``; ``total_it`` stays.
* ``TD3_base.save / load`` (TD3_base.py:26-50) for the particle learner: the reference's six files
  with its key layout (``conv1.weight`` [256, 1, 1, D], ``conv2.weight`` [128, 256, 1],
  ``lnorm1.*``), files written by torch itself, and save -> load -> step bitwise.
* ``ReplayBuffer_particles.save / load`` (my_replay_buffer.py:28-44) round trip.
Tolerances as tests/test_gpu_parity.py.
"""
import contextlib
import copy
import os
import pickle
from collections import OrderedDict

import numpy as np
import pytest

from helpers import gen, orc, particle_setup
from test_gpu_parity import _load_oracle_state, _params_close, _rel_to_max
from test_gpu_particles import _make

pytestmark = pytest.mark.gpu


def _states(S, n, seed):
    rs = np.random.RandomState(seed)
    f = rs.standard_normal((n, S["F"])).astype(np.float32)
    p = rs.standard_normal((n, S["N"], S["D"])).astype(np.float32)
    return f, p


@contextlib.contextmanager
def _oracle_f64():
    """The oracle's arithmetic in float64 (its dtype is the module's ``f32`` alias): the exact
    reference value against which the GPU's and the float32 oracle's rounding are both measured."""
    old = orc.f32, orc.LN_EPS
    orc.f32, orc.LN_EPS = np.float64, np.float64(1e-5)
    try:
        yield
    finally:
        orc.f32, orc.LN_EPS = old


def _as_f64(L):
    """A copy of oracle learner ``L`` whose parameters, targets and Adam moments are float64."""
    L64 = copy.deepcopy(L)
    for d in (L64.actor, L64.actor_m, L64.actor_v, L64.actor_target,
              L64.critic, L64.critic_m, L64.critic_v, L64.critic_target):
        for k in d:
            d[k] = np.asarray(d[k], dtype=np.float64)
    return L64


def _oracle_after(S, steps, seed):
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(seed)
    for _ in range(steps):
        idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
        noise = rs.standard_normal((S["B"], S["A"])).astype(np.float32)
        orc.particle_train_step(L, S["buf"].gather(idx), noise)
    return L, rs


@pytest.mark.parametrize("name", ["part_layer", "part_nocdq", "part_none"])
def test_actor_learn_matches_oracle(name):
    """Teacher-forced: from the oracle's state after 3 train steps, _actor_learn on 32 fresh
    states (torch tensors, as evaluate_model.py builds them) twice, against the oracle."""
    import torch
    S = particle_setup(name)
    pol, _ = _make(S)
    L, _ = _oracle_after(S, 3, 7)
    for k in range(2):
        _load_oracle_state(pol, L)
        f, p = _states(S, 32, 100 + k)
        L64 = _as_f64(L)
        with _oracle_f64():
            orc.particle_actor_learn(L64, f.astype(np.float64), p.astype(np.float64))
        rec = orc.particle_actor_learn(L, f, p)
        loss = pol._actor_learn(torch.from_numpy(f), torch.from_numpy(p), stats=True)
        np.testing.assert_allclose(loss, rec["actor_loss"], rtol=1e-5, atol=1e-7)
        _params_close(pol.actor.numpy_dict(), L.actor, L.lr, (k, "actor"))
        _params_close(pol.actor_target.numpy_dict(), L.actor_target, L.lr, (k, "actor_target"))
        _params_close(pol.critic_target.numpy_dict(), L.critic_target, L.lr, (k, "critic_target"))
        for kk, v in pol.critic.numpy_dict().items():          # the critic is only read
            np.testing.assert_array_equal(v, L.critic[kk])
        assert pol._counters() == (L.total_it, L.critic_step, L.actor_step)
        # exp_avg = 0.9 m + 0.1 g carries the actor gradient, the end of a 7-stage backward chain
        # (Q1 backward, dQ1/da, tanh, actor MLP, encoder): measured against the float64 oracle, the
        # GPU's error is at most 3x the float32 oracle's own (or 2e-4 of the tensor's scale)
        sd = pol.actor_optimizer.state_dict()
        for i, kk in enumerate(L.actor):
            gpu, ref = sd["state"][i]["exp_avg"].numpy(), L64.actor_m[kk]
            e_gpu, e_orc = _rel_to_max(gpu, ref), _rel_to_max(L.actor_m[kk], ref)
            assert e_gpu <= max(3 * e_orc, 2e-4), (kk, e_gpu, e_orc)


def test_actor_learn_between_train_steps():
    """_actor_learn interleaved with train (batch sizes differ: a plan rebuild each call) leaves
    the learner exactly where the oracle doing the same calls is; total_it counts train only."""
    S = particle_setup("part_layer")
    pol, rb = _make(S)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(3)
    for k in range(3):
        idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
        noise = rs.standard_normal((S["B"], S["A"])).astype(np.float32)
        _load_oracle_state(pol, L)
        rec = orc.particle_train_step(L, S["buf"].gather(idx), noise)
        out = pol.train_step(rb, S["B"], indices=idx, noise=noise, stats=True)
        assert _rel_to_max(out["y"], rec["y"]) <= 1e-5
        _load_oracle_state(pol, L)
        f, p = _states(S, 8, 50 + k)
        orc.particle_actor_learn(L, f, p)
        pol._actor_learn(f, p)
        _params_close(pol.actor.numpy_dict(), L.actor, L.lr, (k, "actor"))
        _params_close(pol.critic_target.numpy_dict(), L.critic_target, L.lr, (k, "critic_target"))
        assert pol.total_it == L.total_it == k + 1
        assert pol._counters()[2] == L.actor_step


def _torch_load(path):
    import torch
    return torch.load(path, map_location="cpu", weights_only=True)


def test_particle_save_writes_reference_files(tmp_path):
    S = particle_setup("part_layer")
    pol, rb = _make(S)
    for _ in range(2):
        pol.train(rb, S["B"])
    pol.save(str(tmp_path))
    names = ["critic", "critic_target", "critic_optimizer", "actor", "actor_target", "actor_optimizer"]
    assert sorted(os.listdir(tmp_path)) == sorted(names)
    D = S["D"]
    for grp, ref in (("actor", S["actor"]), ("critic", S["critic"])):
        sd = _torch_load(tmp_path / grp)
        assert list(sd.keys()) == list(ref.keys()), grp
        for k, v in sd.items():
            assert tuple(v.shape) == ref[k].shape, k
        pre = "q1." if grp == "critic" else ""
        assert tuple(sd[pre + "conv1.weight"].shape) == (256, 1, 1, D)     # Conv2d(1, 256, (1, D))
        assert tuple(sd[pre + "conv2.weight"].shape) == (128, 256, 1)      # Conv1d(256, 128, 1)
        assert pre + "lnorm1.weight" in sd
    actor = _torch_load(tmp_path / "actor")
    for k, v in pol.actor.numpy_dict().items():
        np.testing.assert_array_equal(actor[k].numpy(), v)
    opt = _torch_load(tmp_path / "critic_optimizer")
    assert float(opt["state"][0]["step"]) == 2.0 and len(opt["state"]) == len(S["critic"])
    assert float(_torch_load(tmp_path / "actor_optimizer")["state"][0]["step"]) == 1.0


def test_particle_load_torch_written_checkpoint_then_step(tmp_path):
    """Files written by torch (module tensors + a stepped torch.optim.Adam) load into the particle
    learner, which then continues like the oracle continuing from the same state."""
    import torch
    S = particle_setup("part_layer")
    L, rs = _oracle_after(S, 3, 21)
    for grp, params, m, v, step in (("actor", L.actor, L.actor_m, L.actor_v, L.actor_step),
                                    ("critic", L.critic, L.critic_m, L.critic_v, L.critic_step)):
        ts = OrderedDict((k, torch.nn.Parameter(torch.from_numpy(p.copy()))) for k, p in params.items())
        opt = torch.optim.Adam(list(ts.values()), lr=L.lr)
        for k, p in ts.items():
            opt.state[p] = {"step": torch.tensor(float(step)), "exp_avg": torch.from_numpy(m[k].copy()),
                            "exp_avg_sq": torch.from_numpy(v[k].copy())}
        torch.save(OrderedDict((k, t.detach()) for k, t in ts.items()), tmp_path / grp)
        tgt = L.actor_target if grp == "actor" else L.critic_target
        torch.save(OrderedDict((k, torch.from_numpy(t.copy())) for k, t in tgt.items()), tmp_path / f"{grp}_target")
        torch.save(opt.state_dict(), tmp_path / f"{grp}_optimizer")
    pol, rb = _make(S)
    pol.load(str(tmp_path))
    assert pol._counters()[1:] == (L.critic_step, L.actor_step)
    pol.total_it = L.total_it
    for k, x in pol.critic.numpy_dict().items():
        np.testing.assert_array_equal(x, L.critic[k], err_msg=k)
    idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
    noise = rs.standard_normal((S["B"], S["A"])).astype(np.float32)
    rec = orc.particle_train_step(L, S["buf"].gather(idx), noise)
    out = pol.train_step(rb, S["B"], indices=idx, noise=noise, stats=True)
    assert out["actor_step"] and _rel_to_max(out["y"], rec["y"]) <= 1e-5
    _params_close(pol.actor.numpy_dict(), L.actor, L.lr, "actor")
    _params_close(pol.critic.numpy_dict(), L.critic, L.lr, "critic")
    _params_close(pol.critic_target.numpy_dict(), L.critic_target, L.lr, "critic_target")


def test_particle_save_load_resume_is_bitwise(tmp_path):
    S = particle_setup("part_layer")
    a, rb = _make(S)
    for _ in range(3):
        a.train(rb, S["B"])
    a.save(str(tmp_path))
    b, _ = _make(S)
    b.load(str(tmp_path))
    b.total_it = a.total_it
    rs = np.random.RandomState(5)
    for _ in range(2):
        idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
        noise = rs.standard_normal((S["B"], S["A"])).astype(np.float32)
        a.train_step(rb, S["B"], indices=idx, noise=noise)
        b.train_step(rb, S["B"], indices=idx, noise=noise)
    for va, vb in ((a.actor, b.actor), (a.critic, b.critic), (a.actor_target, b.actor_target),
                   (a.critic_target, b.critic_target)):
        np.testing.assert_array_equal(va.flat(), vb.flat())


def test_particle_replay_buffer_files_roundtrip(tmp_path):
    from td3_amd.my_replay_buffer import ReplayBuffer_particles
    from test_gpu_parity import Box
    F, N, D, A, cap = 3, 5, 4, 2, 16
    obs = (Box((F,)), Box((N, D)))
    rb = ReplayBuffer_particles(obs, Box((A,)), max_size=cap)
    rs = np.random.RandomState(4)
    n = 21                                             # wraps: ptr = 5, size = 16
    f, p = rs.standard_normal((n, F)), rs.standard_normal((n, N, D))
    a, f2, p2 = rs.uniform(-1, 1, (n, A)), rs.standard_normal((n, F)), rs.standard_normal((n, N, D))
    r, d = rs.standard_normal(n), (rs.uniform(size=n) < 0.3).astype(np.float64)
    for i in range(n):
        rb.add((f[i], p[i]), a[i], (f2[i], p2[i]), r[i], d[i])
    rb.save(str(tmp_path))
    with open(tmp_path / "ptr.pkl", "rb") as fh:
        assert pickle.load(fh) == 5
    with open(tmp_path / "size.pkl", "rb") as fh:
        assert pickle.load(fh) == 16
    with open(tmp_path / "state_particles.pkl", "rb") as fh:
        arr = np.load(fh)
    assert arr.dtype == np.float64 and arr.shape == (cap, N, D)
    ring = np.empty_like(arr)
    ring[:5] = p[16:21]
    ring[5:] = p[5:16]
    np.testing.assert_array_equal(arr, ring.astype(np.float32).astype(np.float64))
    rb2 = ReplayBuffer_particles(obs, Box((A,)), max_size=cap, load_folder=str(tmp_path))
    assert (rb2.ptr, rb2.size) == (5, 16)
    idx = np.arange(cap)
    for x, y in zip(rb.sample(cap, indices=idx), rb2.sample(cap, indices=idx)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
