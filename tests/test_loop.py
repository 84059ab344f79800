"""Host side of the acting loop: OU noise, loop order and the
batched hindsight add.  CPU only: the learner and buffer are recording fakes."""
import numpy as np

from td3_amd.exploration import OrnsteinUhlenbeckActionNoise
from td3_amd.loop import SyntheticEnv, TrainLoop, add_to_replay_buffer


def test_ou_noise_matches_reference_recurrence():
    """utils/noise.py:17-21: dx = theta (mu - X); dx += sigma randn; X += dx (float64)."""
    np.random.seed(3)
    ou = OrnsteinUhlenbeckActionNoise(4, sigma=0.3)
    got = [ou.sample().copy() for _ in range(50)]
    np.random.seed(3)
    X = np.ones(4) * 0
    for g in got:
        dx = 0.1 * (0 - X)
        dx = dx + 0.3 * np.random.randn(4)
        X = X + dx
        np.testing.assert_array_equal(g, X)
    ou.reset()
    np.testing.assert_array_equal(ou.X, np.zeros(4))


class FakePolicy:
    def __init__(self, ad):
        self.ad, self.log = ad, []

    def select_action(self, s):
        self.log.append("act")
        return np.full(self.ad, 0.25)

    def train(self, rb, b):
        self.log.append(("train", b, len(rb.rows)))


class FakeBuffer:
    def __init__(self):
        self.rows, self.calls = [], 0

    def add(self, s, a, s2, r, d):
        self.calls += 1
        self.rows.append((np.asarray(s), np.asarray(a), np.asarray(s2), float(r), float(d)))

    def add_batch(self, s, a, s2, r, d):
        self.calls += 1
        for i in range(len(r)):
            self.rows.append((s[i], a[i], s2[i], float(r[i]), float(d[i])))


def test_loop_order_follows_main():
    env = SyntheticEnv(5, 2, max_action=1.0, max_episode_steps=7)
    pol, rb = FakePolicy(2), FakeBuffer()
    ends = []
    loop = TrainLoop(env, pol, rb, max_action=1.0, start_policy=4, start_training=6, batch_size=32,
                     expl_noise=0.1, on_episode_end=ends.append)
    np.random.seed(0)
    r = loop.run(20)
    assert r["grad_steps"] == 14 and r["episodes"] == 2
    # no select_action before start_policy; train after the add of the same step
    assert pol.log[0] == "act" and pol.log.count("act") == 16
    trains = [x for x in pol.log if x != "act"]
    assert [x[2] for x in trains] == list(range(7, 21))
    assert all(x[1] == 32 for x in trains)
    # done_swap: the time-limit end of an episode is stored as not done
    assert [row[4] for row in rb.rows[:7]] == [0.0] * 7
    assert [e["length"] for e in ends] == [7, 7]
    # actions are clipped to max_action
    assert max(np.abs(row[1]).max() for row in rb.rows) <= 1.0


def test_hindsight_relabels_are_one_batched_add():
    rb = FakeBuffer()
    s, s2 = np.arange(3.0), np.arange(3.0) + 1
    rel = [(s * 2, s2 * 2, 5.0), (s * 3, s2 * 3, 6.0)]
    add_to_replay_buffer(rb, s, np.array([0.5]), 1.0, s2, 0.0, rel)
    assert rb.calls == 1 and len(rb.rows) == 3
    np.testing.assert_array_equal(rb.rows[2][0], s * 3)
    assert [row[3] for row in rb.rows] == [1.0, 5.0, 6.0]
    assert all(row[1][0] == 0.5 for row in rb.rows)
    add_to_replay_buffer(rb, s, np.array([0.5]), 1.0, s2, 1.0)
    assert rb.calls == 2 and rb.rows[-1][4] == 1.0
