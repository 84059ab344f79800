#!/usr/bin/env python3
"""Where the time of a short timed run goes (GPU box diagnostic, not product code): the driver's bench
form (20 steps after 5 warm-up) timed on the host clock as bench.py does, and on the GPU clock by two
HIP events on the learner stream around the same steps."""
import ctypes as C
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
    steps = int(os.environ.get("SP_STEPS", "20"))
    pol = TD3(Box((17,)), Box((6,)), max_action=1.0, device=0, seed=17, use_graph="auto")
    rb = RB(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=101)
    rb.fill_synthetic(1_000_000, 1.0, seed=7)
    for _ in range(5):
        pol.train(rb, 256)
    stream = torch.cuda.ExternalStream(int(pol._lib.td3_stream(pol._h)), device=0)
    for rep in range(8):
        pol.sync()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        t1 = time.perf_counter()
        for _ in range(steps):
            pol.train(rb, 256)
        t2 = time.perf_counter()
        e1.record(stream)
        pol.sync()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        gpu = e0.elapsed_time(e1) * 1e3
        print(f"run {rep}: host {1e6 * (t4 - t0):7.1f} us (enqueue {1e6 * (t2 - t1):6.1f}, sync {1e6 * (t3 - t2):6.1f}, "
              f"torch sync {1e6 * (t4 - t3):5.1f})  gpu events {gpu:7.1f} us = {gpu / steps:6.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
