"""Pin the torch-CPU restatement (oracle/td3_torch_cpu.py, bench.py's cpu_baseline) against the
goldens the reference itself produced (tests/golden/make_golden.py): every step free-running
from the same initial state with the recorded indices and noise."""
import numpy as np
import pytest

from helpers import gen, load_golden, featured_setup, particle_setup
from test_oracle_golden import _rel_to_max

from oracle.td3_torch_cpu import FeaturedTorch, ParticleTorch


def _check_params(T, G, p, atol):
    for grp, sb in (("actor", 0), ("critic", 500), ("actor_target", 0), ("critic_target", 500)):
        for i, (k, v) in enumerate(T.numpy(grp).items()):
            _, smp = gen.summarize(v, salt=sb + i)
            assert np.abs(smp - G[f"{p}/{grp}/{k}/samples"]).max() <= atol, (p, grp, k)


@pytest.mark.parametrize("name", ["pend_layer", "hc_layer", "hc_none", "hc_layer_hp", "hum_layer"])
def test_featured_torch_restatement_matches_reference(name):
    G = load_golden("featured", name)
    S = featured_setup(name)
    T = FeaturedTorch(S["actor"], S["critic"], **S["kw"])
    for step in range(1, S["steps"] + 1):
        p = f"step{step}"
        rec = T.train_step(S["buf"].gather(G[f"{p}/idx"]), G[f"{p}/noise"])
        for k in ("y", "q1", "q2"):
            assert _rel_to_max(rec[k], G[f"{p}/{k}"]) <= 2e-5, (p, k)
        np.testing.assert_allclose(rec["critic_loss"], G[f"{p}/critic_loss"], rtol=1e-5)
        assert bool(G[f"{p}/actor_step"]) == ("actor_loss" in rec)
        if "actor_loss" in rec:
            np.testing.assert_allclose(rec["actor_loss"], G[f"{p}/actor_loss"], rtol=1e-5)
        _check_params(T, G, p, 2e-5)


@pytest.mark.parametrize("name", list(gen.PARTICLE_CONFIGS))
def test_particle_torch_restatement_matches_reference(name):
    G = load_golden("particles", name)
    S = particle_setup(name)
    T = ParticleTorch(S["actor"], S["critic"], **S["kw"])
    for step in range(1, S["steps"] + 1):
        p = f"step{step}"
        rec = T.train_step(S["buf"].gather(G[f"{p}/idx"]), G[f"{p}/noise"])
        for k in ("y", "q1"):
            assert _rel_to_max(rec[k], G[f"{p}/{k}"]) <= 2e-5, (p, k)
        np.testing.assert_allclose(rec["critic_loss"], G[f"{p}/critic_loss"], rtol=1e-5)
        if "actor_loss" in rec:
            np.testing.assert_allclose(rec["actor_loss"], G[f"{p}/actor_loss"], rtol=1e-5)
        _check_params(T, G, p, 5e-5)
