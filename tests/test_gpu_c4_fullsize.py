"""BASELINE configuration C4 at its real size on the MI355X: ``TD3_particles.train`` at F=7,
N=350, D=9, A=3, B=4096 (/root/reference/TD3_particles.py:167-224) on a 1e5-row
ring filled on the device (25 GB of particle records).

Two production steps (Philox rows over the whole ring, device noise) -- a critic-only step and a
policy step -- read back the rows and noise they drew; the oracle replays the same steps on the
same records, teacher-forced, at the SURVEY §8c tolerances.  This is the only test that runs the
B=4096 variants of the particle learner: the 128-column GEMM stages, the 64x64 LDS-DMA dW tiles
with the lnorm1 LayerNorm-only problem, the A-output Q heads and the 256-workgroup encoder
backward over 4096 rows x 11 particle tiles.  The oracle needs ~10-20 s per step here.
"""
import numpy as np
import pytest

from helpers import gen, orc
from test_gpu_parity import _load_oracle_state, _params_close, _rel_to_max

pytestmark = pytest.mark.gpu

F, N, D, A, B, ROWS = 7, 350, 9, 3, 4096, 100_000


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def _batch(rb, idx):
    """The drawn records, read back through the (bit-exact, tests/test_gpu_particles.py) gather."""
    shapes = ((B, F), (B, N, D), (B, A), (B, F), (B, N, D), (B, 1), (B, 1))
    out = rb.sample(B, indices=idx)
    return tuple(t.cpu().numpy().reshape(s).astype(np.float32) for t, s in zip(out, shapes))


@pytest.mark.timeout(900)
def test_c4_full_size_philox_steps_teacher_forced():
    from td3_amd.TD3_particles import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_particles
    actor = gen.init_params(gen.particle_actor_shapes(F, D, A, "layer"), 41)
    critic = gen.init_params(gen.particle_critic_shapes(F, D, A, "layer", True), 42)
    obs = (Box((F,)), Box((N, D)))
    pol = TD3(obs, Box((A,)), norm="layer", CDQ=True, use_graph="auto", init="none", seed=5)
    pol.set_weights(actor, critic)
    rb = ReplayBuffer_particles(obs, Box((A,)), max_size=ROWS, seed=9)
    rb.fill_synthetic(ROWS, 1.0, seed=3)
    assert rb.size == ROWS
    L = orc.Learner(actor, critic, norm="layer", cdq=True)
    for step in (1, 2):
        _load_oracle_state(pol, L)
        out = pol.train_step(rb, B, stats=True)
        idx, noise = out["idx"], out["noise"]
        assert idx.min() >= 0 and idx.max() < ROWS and len(np.unique(idx)) > 0.9 * B
        assert np.isfinite(noise).all() and 0.9 < noise.std() < 1.1
        rec = orc.particle_train_step(L, _batch(rb, idx), noise)
        assert out["actor_step"] == (step == 2) == ("actor_loss" in rec)
        assert _rel_to_max(out["y"], rec["y"]) <= 1e-5, (step, "y")
        assert _rel_to_max(out["q1"], rec["q1"]) <= 1e-5, (step, "q1")
        assert _rel_to_max(out["q2"], rec["q2"]) <= 1e-5, (step, "q2")
        np.testing.assert_allclose(out["critic_loss"], rec["critic_loss"], rtol=1e-5)
        if out["actor_step"]:
            np.testing.assert_allclose(out["actor_loss"], rec["actor_loss"], rtol=1e-5, atol=1e-7)
        _params_close(pol.critic.numpy_dict(), L.critic, L.lr, (step, "critic"))
        _params_close(pol.critic_target.numpy_dict(), L.critic_target, L.lr, (step, "critic_target"))
        _params_close(pol.actor.numpy_dict(), L.actor, L.lr, (step, "actor"))
        _params_close(pol.actor_target.numpy_dict(), L.actor_target, L.lr, (step, "actor_target"))
        assert pol._counters() == (L.total_it, L.critic_step, L.actor_step)
