#!/usr/bin/env python3
"""Host-submission probe: is the train() loop host-bound?  (GPU box helper, not a test.)

Prints, for the bench workload: wall steps/s, host-only submission time per step (loop
without sync), and the same loop calling the C-ABI directly (no Python wrapper).
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (single HIP runtime: torch first)

from td3_amd.TD3_featured import TD3  # noqa: E402
from td3_amd.my_replay_buffer import ReplayBuffer_featured  # noqa: E402


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    graph = os.environ.get("PROBE_EAGER", "0") != "1"
    pol = TD3(Box((17,)), Box((6,)), max_action=1.0, norm="layer", device=0, seed=1, use_graph=graph)
    rb = ReplayBuffer_featured(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=2)
    rb.fill_synthetic(1_000_000, 1.0, seed=3)
    for _ in range(50):
        pol.train(rb, 256)
    pol.sync()
    t0 = time.perf_counter()
    for _ in range(n):
        pol.train(rb, 256)
    th = time.perf_counter() - t0
    pol.sync()
    tw = time.perf_counter() - t0
    print(f"python loop: wall {n / tw:.1f} steps/s ({tw / n * 1e6:.1f} us/step), host submit {th / n * 1e6:.1f} us/step")
    lib, h, rh = pol._lib, pol._h, rb.handle
    t0 = time.perf_counter()
    for _ in range(n):
        lib.td3_train_step(h, rh, 256, None, None, None, None)
    th = time.perf_counter() - t0
    pol.sync()
    tw = time.perf_counter() - t0
    print(f"ctypes loop: wall {n / tw:.1f} steps/s ({tw / n * 1e6:.1f} us/step), host submit {th / n * 1e6:.1f} us/step")


if __name__ == "__main__":
    main()
