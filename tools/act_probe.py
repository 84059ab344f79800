#!/usr/bin/env python3
"""select_action host-time split (GPU box helper, not product code): the Python wrapper, the bare
C call with cached pointers, and the query launches alone; run under rocprofv3 --kernel-trace
--stats for the kernels' durations.  HalfCheetah shapes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, n=3000):
    for _ in range(100):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from td3_amd import _lib
    from td3_amd.TD3_featured import TD3
    from td3_amd.loop import SyntheticEnv
    sd, ad = 17, 6
    env = SyntheticEnv(sd, ad, max_action=1.0)
    pol = TD3(env.observation_space, env.action_space, max_action=1.0, norm="layer")
    s = env.reset().astype(np.float32)
    out = np.empty(ad, np.float32)
    ps, po = _lib.fptr(s), _lib.fptr(out)
    lib, h = pol._lib, pol._h
    print(f"{'select_action (python API)':40s} {timeit(lambda: pol.select_action(s)):8.1f} us")
    print(f"{'td3_select_action (cached ctypes)':40s} {timeit(lambda: lib.td3_select_action(h, ps, po, 1)):8.1f} us")
    s4 = np.tile(s, (4, 1))
    o4 = np.empty((4, ad), np.float32)
    p4, q4 = _lib.fptr(s4), _lib.fptr(o4)
    print(f"{'td3_select_action n=4':40s} {timeit(lambda: lib.td3_select_action(h, p4, q4, 4)):8.1f} us")
    s32 = np.tile(s, (32, 1))
    o32 = np.empty((32, ad), np.float32)
    p32, q32 = _lib.fptr(s32), _lib.fptr(o32)
    print(f"{'td3_select_action n=32 (GEMM stages)':40s} {timeit(lambda: lib.td3_select_action(h, p32, q32, 32)):8.1f} us")
    print(f"{'td3_last_error (bare ctypes call)':40s} {timeit(lambda: lib.td3_last_error()):8.1f} us")


if __name__ == "__main__":
    main()
