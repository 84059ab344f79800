"""Edge cases of the HIP step against the oracle (teacher-forced, SURVEY.md §8c tolerances).

* ragged batches: B = 1, 33, 257 (row tiles of 32 with 31 / 31 / 31 padding rows), and the
  64x64 dW tiles of B >= 512: B = 544 (Bp % 64 = 32: register-staged dw64_kernel) and B = 640
  (LDS-DMA dw64g_kernel, whose 64-row steps need Bp % 64 = 0; edge tiles with dead quadrants);
* hidden widths other than the reference's (500, 400, 300) / (500, 400, 200): narrow, odd and
  the 512-wide maximum (every Linear / LayerNorm is padded to 32 in HBM, td3.hip);
* the widest action space the heads take (32) and the widest network input (512 columns, a
  record too wide for the sample fused into the first layer: the separate gather kernel);
* an empty ring (the reference's ``np.random.randint(0, 0)`` raises; so does the library) and a
  bulk add of more rows than the capacity (``my_replay_buffer.py:115-116`` applied n times).

Widths and dims here have no reference golden: the oracle (pinned to the reference by
tests/test_oracle_golden.py on the golden configs) is the checker.
"""
import numpy as np
import pytest

from helpers import gen, orc
from test_gpu_parity import Box, _params_close, _load_oracle_state, _rel_to_max

pytestmark = pytest.mark.gpu


def _setup(sd, ad, ma=1.0, norm="layer", actor_arch=gen.ACTOR_ARCH, q_arch=gen.Q_ARCH, rows=gen.BUFFER_ROWS):
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    a0 = gen.init_params(gen._mlp_shapes("", sd, actor_arch, ad, norm), gen.SEED)
    c0 = gen.init_params(gen._mlp_shapes("q1.", sd + ad, q_arch, 1, norm) +
                         gen._mlp_shapes("q2.", sd + ad, q_arch, 1, norm), gen.SEED + 100)
    buf = orc.FeaturedBuffer(sd, ad, rows)
    s, a, s2, r, d = gen.fill_featured_buffer(sd, ad, ma, rows, gen.SEED)
    for i in range(rows):
        buf.add(s[i], a[i], s2[i], r[i], d[i])
    pol = TD3(Box((sd,)), Box((ad,)), max_action=ma, norm=norm, actor_arch=actor_arch, q_arch=q_arch,
              init="none")
    pol.set_weights(a0, c0)
    rb = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=rows)
    rb.add_batch(s, a, s2, r, d)
    L = orc.Learner(a0, c0, max_action=ma, norm=norm)
    return pol, rb, L, buf


def _teacher_forced(pol, rb, L, buf, B, ad, seed, steps=2):
    rs = np.random.RandomState(seed)
    for step in range(1, steps + 1):
        idx = rs.randint(0, buf.size, B)
        noise = rs.standard_normal((B, ad)).astype(np.float32)
        _load_oracle_state(pol, L)
        rec = orc.featured_train_step(L, buf.gather(idx), noise)
        out = pol.train_step(rb, B, indices=idx, noise=noise, stats=True)
        np.testing.assert_array_equal(out["idx"], idx)
        assert _rel_to_max(out["y"], rec["y"][:, 0]) <= 1e-5, (step, "y")
        assert _rel_to_max(out["q1"], rec["q1"][:, 0]) <= 1e-5, (step, "q1")
        assert _rel_to_max(out["q2"], rec["q2"][:, 0]) <= 1e-5, (step, "q2")
        np.testing.assert_allclose(out["critic_loss"], rec["critic_loss"], rtol=1e-5)
        assert out["actor_step"] == ("actor_loss" in rec)
        if out["actor_step"]:
            np.testing.assert_allclose(out["actor_loss"], rec["actor_loss"], rtol=1e-5, atol=1e-7)
        _params_close(pol.critic.numpy_dict(), L.critic, L.lr, (step, "critic"))
        _params_close(pol.actor.numpy_dict(), L.actor, L.lr, (step, "actor"))
        _params_close(pol.critic_target.numpy_dict(), L.critic_target, L.lr, (step, "critic_target"))
        _params_close(pol.actor_target.numpy_dict(), L.actor_target, L.lr, (step, "actor_target"))


@pytest.mark.parametrize("B", [1, 33, 257])
def test_ragged_batches(B):
    pol, rb, L, buf = _setup(17, 6)
    _teacher_forced(pol, rb, L, buf, B, 6, seed=B)


@pytest.mark.parametrize("B", [544, 640])
def test_large_batch_dw_tiles(B):
    pol, rb, L, buf = _setup(17, 6)
    _teacher_forced(pol, rb, L, buf, B, 6, seed=B)


@pytest.mark.parametrize("norm", ["layer", None])
def test_custom_hidden_widths(norm):
    pol, rb, L, buf = _setup(11, 3, norm=norm, actor_arch=(64, 48, 40), q_arch=(96, 72, 33))
    _teacher_forced(pol, rb, L, buf, 96, 3, seed=5)


def test_widest_hidden_layers():
    pol, rb, L, buf = _setup(17, 6, actor_arch=(512, 512, 512), q_arch=(512, 512, 512))
    _teacher_forced(pol, rb, L, buf, 128, 6, seed=6)


def test_widest_action_space():
    pol, rb, L, buf = _setup(9, 32, ma=0.5)
    _teacher_forced(pol, rb, L, buf, 64, 32, seed=7)


def test_widest_network_input():
    """sd + ad = 512: the critic's first Linear takes the widest input the GEMM stages handle; the
    record (994 floats) is sampled by the separate gather kernel."""
    pol, rb, L, buf = _setup(480, 32, ma=0.4, rows=300)
    _teacher_forced(pol, rb, L, buf, 64, 32, seed=8)


def test_empty_ring_raises():
    from td3_amd import _lib
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    pol = TD3(Box((5,)), Box((2,)), init="none")
    rb = ReplayBuffer_featured(Box((5,)), Box((2,)), max_size=10)
    with pytest.raises(_lib.TD3Error, match="empty"):
        pol.train(rb, 4)
    with pytest.raises(_lib.TD3Error, match="empty"):
        rb.sample(4)


def test_bulk_add_past_capacity():
    """130 rows into a 50-row ring in one add: the last 50 survive, ptr = 130 % 50, size = 50,
    exactly as 130 single adds (my_replay_buffer.py:109-117)."""
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    sd, ad, cap, n = 7, 2, 50, 130
    s, a, s2, r, d = gen.fill_featured_buffer(sd, ad, 1.0, n, 11)
    ref = orc.FeaturedBuffer(sd, ad, cap)
    for i in range(n):
        ref.add(s[i], a[i], s2[i], r[i], d[i])
    rb = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=cap)
    rb.add_batch(s[:3], a[:3], s2[:3], r[:3], d[:3])          # ptr starts mid-ring
    rb.add_batch(s[3:], a[3:], s2[3:], r[3:], d[3:])
    assert (rb.ptr, rb.size) == (ref.ptr, ref.size) == (n % cap, cap)
    idx = np.arange(cap)
    for got, want in zip(rb.sample(cap, indices=idx), ref.gather(idx)):
        np.testing.assert_array_equal(got.cpu().numpy(), np.asarray(want, np.float32))
