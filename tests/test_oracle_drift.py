"""The oracle over 100 free-running steps against the reference's own run (CPU).

``tests/golden/drift_hc_layer.npz`` (``make_drift.py``) holds 100 reference ``TD3.train`` steps
(HalfCheetah dims, B = 256, LayerNorm; ``TD3_featured.py:123-171`` as ``main.py:266-269`` calls
it) and the envelope of the reference's own fp32 drift: the reference against itself at 1 vs
2 / 4 / 8 torch threads.  SURVEY.md §8c: free-running drift must stay inside that envelope.
This pins the oracle over the long horizon; ``test_gpu_drift.py`` holds the HIP path to the
same contract.
"""
import numpy as np

from helpers import drift_check, drift_envelope, featured_setup_dims, gen, load_golden, orc


def test_oracle_free_running_100_steps_inside_reference_envelope():
    G = load_golden("drift", "hc_layer")
    sd, ad, ma, norm, B = gen.DRIFT_CONFIG
    S = featured_setup_dims(sd, ad, ma, norm, B)
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    env = drift_envelope(G)
    assert env[0] < 1e-7 and env[-1] > 1e-4          # the fixture really drifts
    worst = 0.0
    for step in range(1, gen.DRIFT_STEPS + 1):
        idx, noise = gen.drift_draws(step, B, ad, gen.BUFFER_ROWS)
        orc.featured_train_step(L, S["buf"].gather(idx), noise)
        groups = [("actor", L.actor), ("critic", L.critic)]
        if step in G["target_steps"]:
            groups += [("actor_target", L.actor_target), ("critic_target", L.critic_target)]
        for g, P in groups:
            d, ratio = drift_check(G, step, g, P, env)
            assert ratio <= 1.0, (step, g, d, env[step - 1])
            worst = max(worst, ratio)
    assert L.total_it == gen.DRIFT_STEPS
    print(f"oracle drift / reference envelope, worst over 100 steps: {worst:.3f}")
