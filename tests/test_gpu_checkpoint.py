"""Checkpoint interop on the MI355X.

* TD3_base.save writes the reference's six files as torch state_dicts (TD3_base.py:26-34):
  reference key layout, torch.optim.Adam state format;
* TD3_base.load reads files written by torch itself (a torch.optim.Adam that has stepped), and
  the learner then continues exactly like the oracle continuing from the same state;
* save -> load -> one step is bitwise the step the saved learner takes;
* ReplayBuffer save / load use the reference's file set (my_replay_buffer.py:91-107):
  ``ptr.pkl`` / ``size.pkl`` (pickled ints) and ``<attr>.pkl`` files holding ``np.save``
  float64 arrays.  Only files written here are read back (our own pickles).
"""
import os
import pickle
from collections import OrderedDict

import numpy as np
import pytest

from helpers import gen, orc, featured_setup
from test_gpu_parity import _make, _params_close, _load_oracle_state, _rel_to_max

pytestmark = pytest.mark.gpu


def _torch_load(path):
    import torch
    return torch.load(path, map_location="cpu", weights_only=True)


def _oracle_after(S, steps, seed):
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(seed)
    for _ in range(steps):
        idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
        noise = rs.standard_normal((S["B"], S["ad"])).astype(np.float32)
        orc.featured_train_step(L, S["buf"].gather(idx), noise)
    return L, rs


def test_save_writes_reference_files(tmp_path):
    S = featured_setup("hc_layer")
    pol, rb = _make(S)
    for _ in range(2):
        pol.train(rb, S["B"])
    pol.save(str(tmp_path))
    names = ["critic", "critic_target", "critic_optimizer", "actor", "actor_target", "actor_optimizer"]
    assert sorted(os.listdir(tmp_path)) == sorted(names)
    actor = _torch_load(tmp_path / "actor")
    assert list(actor.keys()) == list(S["actor"].keys())
    for k, v in actor.items():
        assert tuple(v.shape) == S["actor"][k].shape, k
        np.testing.assert_array_equal(v.numpy(), pol.actor.numpy_dict()[k])
    critic = _torch_load(tmp_path / "critic")
    assert list(critic.keys()) == list(S["critic"].keys())
    opt = _torch_load(tmp_path / "critic_optimizer")
    assert set(opt) == {"state", "param_groups"}
    assert len(opt["state"]) == len(critic) and float(opt["state"][0]["step"]) == 2.0
    g = opt["param_groups"][0]
    assert g["betas"] == (0.9, 0.999) and g["eps"] == 1e-8 and g["params"] == list(range(len(critic)))
    aopt = _torch_load(tmp_path / "actor_optimizer")
    assert float(aopt["state"][0]["step"]) == 1.0


def test_load_torch_written_checkpoint_then_step(tmp_path):
    """Files produced by torch (modules' tensors + a stepped torch.optim.Adam) load into the
    learner; one more step matches the oracle continuing from the same state."""
    import torch
    S = featured_setup("hc_layer")
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
    pol.total_it = L.total_it          # TD3_base keeps total_it outside the checkpoint (TD3_base.py:24)
    for what, gpu, ref in (("actor", pol.actor, L.actor), ("critic_t", pol.critic_target, L.critic_target)):
        for k, x in gpu.numpy_dict().items():
            np.testing.assert_array_equal(x, ref[k], err_msg=f"{what} {k}")
    idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
    noise = rs.standard_normal((S["B"], S["ad"])).astype(np.float32)
    rec = orc.featured_train_step(L, S["buf"].gather(idx), noise)
    out = pol.train_step(rb, S["B"], indices=idx, noise=noise, stats=True)
    assert out["actor_step"] and _rel_to_max(out["y"], np.ravel(rec["y"])) <= 1e-5
    _params_close(pol.actor.numpy_dict(), L.actor, L.lr, "actor")
    _params_close(pol.critic.numpy_dict(), L.critic, L.lr, "critic")
    _params_close(pol.actor_target.numpy_dict(), L.actor_target, L.lr, "actor_target")


def test_save_load_resume_is_bitwise(tmp_path):
    S = featured_setup("hc_layer")
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
        noise = rs.standard_normal((S["B"], S["ad"])).astype(np.float32)
        a.train_step(rb, S["B"], indices=idx, noise=noise)
        b.train_step(rb, S["B"], indices=idx, noise=noise)
    for va, vb in ((a.actor, b.actor), (a.critic, b.critic), (a.actor_target, b.actor_target),
                   (a.critic_target, b.critic_target)):
        np.testing.assert_array_equal(va.flat(), vb.flat())
    np.testing.assert_array_equal(a.critic_optimizer.state_dict()["state"][3]["exp_avg_sq"].numpy(),
                                  b.critic_optimizer.state_dict()["state"][3]["exp_avg_sq"].numpy())


def test_replay_buffer_files_roundtrip(tmp_path):
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    from test_gpu_parity import Box
    sd, ad, cap = 5, 2, 64
    rb = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=cap)
    rs = np.random.RandomState(2)
    n = 80                                           # wraps: ptr = 16, size = 64
    s, a, s2 = rs.standard_normal((n, sd)), rs.uniform(-1, 1, (n, ad)), rs.standard_normal((n, sd))
    r, d = rs.standard_normal(n), (rs.uniform(size=n) < 0.2).astype(np.float64)
    for i in range(n):
        rb.add(s[i], a[i], s2[i], r[i], d[i])
    rb.save(str(tmp_path))
    with open(tmp_path / "ptr.pkl", "rb") as f:
        assert pickle.load(f) == 16
    with open(tmp_path / "size.pkl", "rb") as f:
        assert pickle.load(f) == 64
    want = {"state": s, "action": a, "next_state": s2, "reward": r.reshape(-1, 1), "not_done": 1 - d.reshape(-1, 1)}
    for k, full in want.items():
        with open(tmp_path / f"{k}.pkl", "rb") as f:
            arr = np.load(f)
        assert arr.dtype == np.float64 and arr.shape == (cap,) + full.shape[1:], k
        ring = np.empty_like(arr)
        ring[:16] = full[64:80]
        ring[16:] = full[16:64]
        np.testing.assert_array_equal(arr, ring.astype(np.float32).astype(np.float64), err_msg=k)
    rb2 = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=cap, load_folder=str(tmp_path))
    assert (rb2.ptr, rb2.size) == (16, 64)
    idx = np.arange(cap)
    for x, y in zip(rb.sample(cap, indices=idx), rb2.sample(cap, indices=idx)):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())


def _reference_save(folder, buf, names):
    """The reference's ``save`` (my_replay_buffer.py:91-99) over an oracle buffer's arrays."""
    os.makedirs(folder, exist_ok=True)
    for attrib in ("ptr", "size"):
        with open(os.path.join(folder, attrib + ".pkl"), "wb") as f:
            pickle.dump(getattr(buf, attrib), f, protocol=4)
    for attrib in names:
        with open(os.path.join(folder, attrib + ".pkl"), "wb") as f:
            np.save(f, getattr(buf, attrib))


def _same_files(a, b, names):
    for n in ("ptr", "size", *names):
        with open(os.path.join(a, n + ".pkl"), "rb") as fa, open(os.path.join(b, n + ".pkl"), "rb") as fb:
            assert fa.read() == fb.read(), n


FEAT = ["state", "action", "next_state", "reward", "not_done"]
PART = ["state_features", "state_particles", "action", "next_state_features", "next_state_particles",
        "reward", "not_done"]


def test_reference_buffer_folder_roundtrips_byte_exact(tmp_path):
    """host_shadow=True: a folder in the reference's format (float64 values an fp32 ring cannot
    hold) loads and saves back byte for byte, and rows added after the load are saved as the
    reference's own add would have stored them (my_replay_buffer.py:101-117)."""
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    from test_gpu_parity import Box
    sd, ad, cap = 5, 2, 64
    rs = np.random.RandomState(4)
    ref = orc.FeaturedBuffer(sd, ad, cap)
    for _ in range(40):
        ref.add(rs.standard_normal(sd), rs.uniform(-1, 1, ad), rs.standard_normal(sd), rs.standard_normal(),
                float(rs.uniform() < 0.2))
    _reference_save(tmp_path / "ref", ref, FEAT)
    rb = ReplayBuffer_featured(Box((sd,)), Box((ad,)), load_folder=str(tmp_path / "ref"), host_shadow=True)
    rb.save(str(tmp_path / "out"))
    _same_files(tmp_path / "ref", tmp_path / "out", FEAT)
    # continue both: single adds and one bulk add that wraps the ring
    for _ in range(10):
        t = (rs.standard_normal(sd), rs.uniform(-1, 1, ad), rs.standard_normal(sd), rs.standard_normal(),
             float(rs.uniform() < 0.2))
        ref.add(*t)
        rb.add(*t)
    n = 30
    bulk = (rs.standard_normal((n, sd)), rs.uniform(-1, 1, (n, ad)), rs.standard_normal((n, sd)),
            rs.standard_normal(n), (rs.uniform(size=n) < 0.2).astype(np.float64))
    for i in range(n):
        ref.add(*(x[i] for x in bulk))
    rb.add_batch(*bulk)
    _reference_save(tmp_path / "ref2", ref, FEAT)
    rb.save(str(tmp_path / "out2"))
    _same_files(tmp_path / "ref2", tmp_path / "out2", FEAT)
    # the training copy is the fp32 ring of the same rows
    idx = np.arange(cap)
    for x, y in zip(rb.sample(cap, indices=idx), ref.gather(idx)):
        np.testing.assert_array_equal(x.cpu().numpy(), y)


def test_reference_particle_buffer_folder_roundtrips_byte_exact(tmp_path):
    from td3_amd.my_replay_buffer import ReplayBuffer_particles
    from test_gpu_parity import Box
    F, N, D, A, cap = 7, 16, 9, 3, 24
    rs = np.random.RandomState(6)
    ref = orc.ParticleBuffer(F, N, D, A, cap)

    def trans():
        return ((rs.standard_normal(F), rs.standard_normal((N, D))), rs.uniform(-1, 1, A),
                (rs.standard_normal(F), rs.standard_normal((N, D))), rs.standard_normal(),
                float(rs.uniform() < 0.2))
    for _ in range(30):                                 # wraps
        ref.add(*trans())
    _reference_save(tmp_path / "ref", ref, PART)
    obs = (Box((F,)), Box((N, D)))
    rb = ReplayBuffer_particles(obs, Box((A,)), load_folder=str(tmp_path / "ref"), host_shadow=True)
    rb.save(str(tmp_path / "out"))
    _same_files(tmp_path / "ref", tmp_path / "out", PART)
    for _ in range(5):
        t = trans()
        ref.add(*t)
        rb.add(*t)
    _reference_save(tmp_path / "ref2", ref, PART)
    rb.save(str(tmp_path / "out2"))
    _same_files(tmp_path / "ref2", tmp_path / "out2", PART)


def test_buffer_without_shadow_after_synthetic_fill_saves_the_ring(tmp_path):
    """A device-only write (fill_synthetic) invalidates the shadow: save falls back to the ring."""
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    from test_gpu_parity import Box
    rb = ReplayBuffer_featured(Box((3,)), Box((1,)), max_size=32, host_shadow=True)
    rb.fill_synthetic(32, 2.0, seed=3)
    rb.save(str(tmp_path))
    with open(tmp_path / "state.pkl", "rb") as f:
        st = np.load(f)
    assert st.dtype == np.float64 and np.abs(st).max() > 0
    np.testing.assert_array_equal(st, st.astype(np.float32).astype(np.float64))
