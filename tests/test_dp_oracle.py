"""The oracle restated in the product's data-parallel form (``helpers.oracle_dp_step``: n replicas
in lock-step threads, each phase's shard gradients summed in replica order and scaled by 1/n before
Adam) against its own global-batch step (CPU).

This is the reference point of the GPU data-parallel tests (tests/test_gpu_data_parallel.py): the
GPU is held to the single-device contract against ``oracle_dp_step``, and to a looser fraction
against the global-batch oracle.  Here the two oracle forms are compared with each other: the
losses and targets agree to fp32 rounding, the gradient is the same up to the order of its fp32 sum,
and the post-Adam parameters differ only where Adam's m / sqrt(v) turns that rounding of a
near-zero gradient into an lr-sized move."""
import numpy as np
import pytest

from helpers import featured_setup, load_golden, oracle_dp_step, orc


def _tight_fraction(a, b):
    fr = []
    for k in b:
        x, y = np.asarray(a[k], np.float64), np.asarray(b[k], np.float64)
        fr.append(np.mean(np.abs(x - y) <= 1e-6 + 1e-5 * np.abs(y)))
    return min(fr)


@pytest.mark.parametrize("name,n", [("hc_layer", 2), ("hc_layer", 4), ("pend_layer", 2)])
def test_dp_oracle_matches_global_batch_oracle(name, n):
    S = featured_setup(name)
    G = load_golden("featured", name)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    lr = S["kw"].get("lr", 1e-4)
    for step in (1, 2):
        batch = S["buf"].gather(G[f"step{step}/idx"])
        noise = G[f"step{step}/noise"]
        Ldp = oracle_dp_step(L, batch, noise, n)
        orc.featured_train_step(L, batch, noise)
        assert (Ldp.total_it, Ldp.critic_step, Ldp.actor_step) == (L.total_it, L.critic_step, L.actor_step)
        for grp in ("critic", "critic_target", "actor", "actor_target"):
            a, b = getattr(Ldp, grp), getattr(L, grp)
            worst = max(float(np.max(np.abs(np.asarray(a[k], np.float64) - b[k]))) for k in b)
            assert worst <= 2 * lr * 1.001, (name, n, step, grp, worst)
            assert _tight_fraction(a, b) >= 0.999, (name, n, step, grp, _tight_fraction(a, b))
        # continue both from the global-batch state (teacher forcing, as the GPU tests)


def test_dp_oracle_replicas_identical_and_one_replica_is_the_oracle():
    """n = 1 is the plain oracle step bit for bit; the replicas of n > 1 end identical."""
    S = featured_setup("pend_layer")
    G = load_golden("featured", "pend_layer")
    batch = S["buf"].gather(G["step1/idx"])
    noise = G["step1/noise"]
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    L1 = oracle_dp_step(L, batch, noise, 1)
    orc.featured_train_step(L, batch, noise)
    for grp in ("critic", "actor", "critic_m", "critic_v"):
        for k, v in getattr(L, grp).items():
            np.testing.assert_array_equal(getattr(L1, grp)[k], v)
