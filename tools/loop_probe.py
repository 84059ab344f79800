#!/usr/bin/env python3
"""Host-time breakdown of one acting-loop iteration (GPU box helper, not product code):
select_action, OU noise, add, train enqueue, each timed over many calls, HalfCheetah shapes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, n=2000):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    from td3_amd.loop import SyntheticEnv
    from td3_amd.exploration import OrnsteinUhlenbeckActionNoise
    sd, ad, ma = 17, 6, 1.0
    env = SyntheticEnv(sd, ad, max_action=ma)
    pol = TD3(env.observation_space, env.action_space, max_action=ma, norm="layer")
    rb = ReplayBuffer_featured(env.observation_space, env.action_space, max_size=1_000_000)
    rb.fill_synthetic(100_000, max_action=ma, seed=1)
    noise = OrnsteinUhlenbeckActionNoise(ad, sigma=0.1)
    s = env.reset()
    a = np.zeros(ad)
    res = {}
    res["select_action (idle GPU)"] = timeit(lambda: pol.select_action(s))
    res["ou noise + clip"] = timeit(lambda: (a + noise.sample()).clip(-ma, ma))
    res["env.step (no busy-wait)"] = timeit(lambda: env.step(a))
    res["rb.add (pending row)"] = timeit(lambda: rb.add(s, a, s, 0.5, 0.0))
    rb.flush()

    def add_flush():
        rb.add(s, a, s, 0.5, 0.0)
        rb.flush()
    res["rb.add + flush (rb_add)"] = timeit(add_flush)
    pol.sync()

    def train_sync():
        pol.train(rb, 256)
        pol.sync()
    res["train + sync (GPU bound)"] = timeit(train_sync, 500)
    t0 = time.perf_counter()
    for _ in range(500):
        pol.train(rb, 256)
    t_enq = (time.perf_counter() - t0) / 500 * 1e6
    pol.sync()
    res["train enqueue, GPU behind (direct launches)"] = t_enq

    def train_after_sync():
        pol.sync()
        t = time.perf_counter()
        pol.train(rb, 256)
        return time.perf_counter() - t
    ts = [train_after_sync() for _ in range(300)]
    res["train enqueue, GPU idle (graph replay)"] = float(np.median(ts)) * 1e6
    for k, v in res.items():
        print(f"{k:45s} {v:8.1f} us")


if __name__ == "__main__":
    main()
