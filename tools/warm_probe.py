#!/usr/bin/env python3
"""Where the driver form's first timed runs lose (GPU box diagnostic, not product code): 5 runs of
20 C2 steps after W warm-up steps, each run timed as bench.py does; WP_PRE = none | spin (a 20 ms
single-wave spin kernel on the torch stream just before the timed runs: the GPU busy, the runtime
and host paths as cold as after 5 steps) | sleep (the host idles 20 ms)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def main():
    import torch
    torch.cuda.set_device(0)
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured as RB
    warm = int(os.environ.get("WP_WARM", "5"))
    pre = os.environ.get("WP_PRE", "none")
    torch.manual_seed(1000)
    pol = TD3(Box((17,)), Box((6,)), max_action=1.0, device=0, seed=17, use_graph="auto")
    rb = RB(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=101)
    rb.fill_synthetic(1_000_000, 1.0, seed=7)
    for _ in range(warm):
        pol.train(rb, 256)
    if pre == "spin":
        pol.sync()
        torch.cuda._sleep(40_000_000)
    elif pre == "sleep":
        pol.sync()
        torch.cuda.synchronize()
        time.sleep(0.02)
    rates = []
    for _ in range(5):
        pol.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            pol.train(rb, 256)
        pol.sync()
        torch.cuda.synchronize()
        rates.append(20 / (time.perf_counter() - t0))
    print(f"warm {warm:5d} pre {pre:5s} runs", [round(r) for r in rates], flush=True)


if __name__ == "__main__":
    main()
