#!/usr/bin/env python3
"""Shader clock of the GEMM stages' MFMA phases in the driver's short runs and in long runs (GPU
box helper, not product code).  Needs the TD3_TL experiment build, whose GEMM
workgroups record s_memtime (shader clock) and s_memrealtime (100 MHz) at the prologue barrier
and at the end of the MFMA loop:

    tools/build_exp.sh tl "-DTD3_TL"
    TD3_LIB=tools/exp/libtd3hip_tl.so python3 tools/clk_probe.py

Runs bench.py's C2 workload (1e6-row ring, B = 256) in the driver's form (5 warm-up steps, then
runs of 20 steps bracketed by syncs) and in 2000-step runs.  Every GEMM workgroup of the run adds
its MFMA phase's shader-clock and 100 MHz tick counts to two device counters (td3_clk_sum): their
ratio x 100 MHz is the clock the run's MFMA phases ran at, weighted by phase length."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def main():
    import torch
    torch.cuda.set_device(0)
    from td3_amd import _lib
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured as RB
    lib = _lib.load()
    for f in (lib.td3_tl_read, lib.td3_clk_read):
        f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_int]
    lib.td3_tl_clear.restype = C.c_int
    torch.manual_seed(1000)
    pol = TD3(Box((17,)), Box((6,)), max_action=1.0, device=0, seed=17, use_graph="auto")
    rb = RB(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=101)
    rb.fill_synthetic(1_000_000, 1.0, seed=7)

    lib.td3_clk_sum_read.restype, lib.td3_clk_sum_read.argtypes = C.c_int, [C.c_void_p, C.c_int]
    acc = np.zeros(2, np.uint64)

    def clock():
        lib.td3_clk_sum_read(acc.ctypes.data, 1)          # read and clear
        return float(acc[0]) / max(float(acc[1]), 1.0) * 100.0

    def timed(steps):
        pol.sync()
        torch.cuda.synchronize()
        clock()
        t0 = time.perf_counter()
        for _ in range(steps):
            pol.train(rb, 256)
        pol.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return steps / dt, clock()

    for _ in range(5):
        pol.train(rb, 256)
    out = {"driver_form": [], "long": []}
    for _ in range(5):
        rate, mhz = timed(20)
        out["driver_form"].append({"steps_s": round(rate, 1), "mfma_mhz": round(mhz)})
    for _ in range(2):
        rate, mhz = timed(2000)
        out["long"].append({"steps_s": round(rate, 1), "mfma_mhz": round(mhz)})
    for _ in range(3):
        rate, mhz = timed(20)
        out["driver_form"].append({"steps_s": round(rate, 1), "mfma_mhz": round(mhz), "after_long": True})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
