"""Diagnostic (GPU box): per-tensor error of the particle learner's actor gradient (through Adam's
exp_avg after one _actor_learn) against the float32 oracle and a float64 run of it."""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
from helpers import particle_setup, orc  # noqa: E402
import test_gpu_particles_api as T  # noqa: E402
from test_gpu_parity import _load_oracle_state  # noqa: E402
from test_oracle_golden import _rel_to_max  # noqa: E402


def run(name, B, call):
    S = particle_setup(name)
    pol, _ = T._make(S)
    L, _ = T._oracle_after(S, 3, 7)
    for kk in range(call):                    # earlier _actor_learn calls (the test's loop)
        f, p = T._states(S, B, 100 + kk)
        orc.particle_actor_learn(L, f, p)
    _load_oracle_state(pol, L)
    f, p = T._states(S, B, 100 + call)
    L64 = T._as_f64(L)
    with T._oracle_f64():
        orc.particle_actor_learn(L64, f.astype(np.float64), p.astype(np.float64))
    orc.particle_actor_learn(L, f, p)
    pol._actor_learn(f, p)
    sd = pol.actor_optimizer.state_dict()
    print(f"== {name} B={B} call {call}")
    for i, k in enumerate(L.actor):
        gpu = sd["state"][i]["exp_avg"].numpy().astype(np.float64)
        ref = L64.actor_m[k]
        e_g, e_o = _rel_to_max(gpu, ref), _rel_to_max(L.actor_m[k], ref)
        d = np.abs(gpu - ref).reshape(gpu.shape[0], -1).max(axis=1) if gpu.ndim > 1 else np.abs(gpu - ref)
        worst = np.argsort(d)[-3:][::-1]
        print(f"{k:22s} gpu {e_g:.2e} orc32 {e_o:.2e}  worst rows {worst.tolist()} {d[worst].tolist()}")


if __name__ == "__main__":
    for k in (0, 1):
        run("part_nocdq", 32, k)
