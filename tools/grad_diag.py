#!/usr/bin/env python3
"""Per-tensor Adam-moment errors against the oracle (GPU box diagnostic, not product code): the
gradient-parity test's two steps at Humanoid widths, printing every tensor's relative error."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from helpers import featured_setup_dims, gen, orc  # noqa: E402
from test_gpu_parity import _load_oracle_state, _make, _rel_to_max  # noqa: E402


def report(opt, m_ref, v_ref, what):
    st = opt.state_dict()["state"]
    bad = []
    for i, k in enumerate(m_ref):
        em = _rel_to_max(st[i]["exp_avg"].numpy(), m_ref[k])
        ev = _rel_to_max(st[i]["exp_avg_sq"].numpy(), v_ref[k])
        flag = "BAD" if em > 1e-4 else ""
        print(f"  {what} {k:28s} m {em:.2e} v {ev:.2e} {flag}")
        if flag:
            bad.append(k)
    return bad


def main():
    B = int(os.environ.get("DIAG_B", "1024"))
    S = featured_setup_dims(376, 17, 0.4, "layer", B=B)
    pol, rb = _make(S, use_graph=not os.environ.get("TD3_DIAG_EAGER"))
    L = orc.Learner(S["actor"], S["critic"], **S["kw"])
    rs = np.random.RandomState(11)
    odd2 = bool(os.environ.get("DIAG_ODD2"))
    for step in (1, 2):
        idx = rs.randint(0, gen.BUFFER_ROWS, size=B)
        if step == 2 and odd2:                  # make step 2 a critic-only step (counters back to 0)
            L.total_it = 0
        noise = rs.standard_normal((B, 17)).astype(np.float32)
        if step == 2:
            _load_oracle_state(pol, L)
        rec = orc.featured_train_step(L, S["buf"].gather(idx), noise)
        out = pol.train_step(rb, B, indices=idx, noise=noise, stats=True)
        print(f"step {step}: y {_rel_to_max(out['y'], rec['y'][:, 0]):.2e} q1 {_rel_to_max(out['q1'], rec['q1'][:, 0]):.2e} "
              f"q2 {_rel_to_max(out['q2'], rec['q2'][:, 0]):.2e}")
        bad = report(pol.critic_optimizer, L.critic_m, L.critic_v, f"critic s{step}")
        if bad and os.environ.get("DIAG_MAP"):
            st = pol.critic_optimizer.state_dict()["state"]
            keys = list(L.critic_m)
            for k in bad[:3]:
                g = st[keys.index(k)]["exp_avg"].numpy().astype(np.float64)
                r = L.critic_m[k].astype(np.float64)
                d = np.abs(g - r) / np.abs(r).max()
                if d.ndim == 2:
                    tn, tk = -(-d.shape[0] // 64), -(-d.shape[1] // 64)
                    m = np.zeros((tn, tk))
                    for a in range(tn):
                        for b in range(tk):
                            m[a, b] = d[64 * a:64 * a + 64, 64 * b:64 * b + 64].max()
                    print(f"  {k} 64x64 tile max err (rows = out blocks):")
                    for a in range(tn):
                        print("   ", " ".join(f"{x:.0e}" for x in m[a]))
                    rows = d.max(axis=1)
                    print("   worst out rows:", np.argsort(-rows)[:8].tolist(), "cols:", np.argsort(-d.max(axis=0))[:8].tolist())


if __name__ == "__main__":
    main()
