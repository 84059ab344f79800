#!/usr/bin/env python3
"""Per-workgroup timeline of the one-launch select_action kernel (GPU box helper, not product
code).  TD3_TL experiment build:  TD3_LIB=tools/exp/libtd3hip_tl.so python3 tools/act_tl.py
Marks (100 MHz s_memrealtime, us from the first workgroup's entry): 5 H0 in LDS, 6 H1 stores
drained, 7 layer-1 poll passed, 1 H2 stores drained, 2 second counter returned, 3 end (the last
arriver: head written and flagged)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from td3_amd import _lib
    from td3_amd.TD3_featured import TD3
    from td3_amd.loop import SyntheticEnv
    lib = _lib.load()
    lib.td3_tl_read.restype, lib.td3_tl_read.argtypes = C.c_int, [C.c_void_p, C.c_int]
    lib.td3_tl_clear.restype = C.c_int
    env = SyntheticEnv(17, 6, max_action=1.0)
    pol = TD3(env.observation_space, env.action_space, max_action=1.0, norm="layer")
    s = env.reset().astype(np.float32)
    for _ in range(50):
        pol.select_action(s)
    rows = []
    for _ in range(20):
        lib.td3_tl_clear()
        pol.select_action(s)
        buf = np.zeros((8192, 8), np.uint64)
        lib.td3_tl_read(buf.ctypes.data, 8192)
        v = buf[buf[:, 0] != 0].astype(np.int64)
        base = v[:, 0].min()
        d = lambda k: (v[:, k][v[:, k] != 0] - base) * 0.01
        rows.append([np.max(d(0)), np.median(d(5)), np.max(d(5)), np.max(d(6)), np.max(d(7)), np.max(d(1)),
                     np.max(d(2)), np.max(d(3)), len(v)])
    r = np.median(np.array(rows), axis=0)
    print("entry_max  H0_p50  H0_max  H1drained_max  poll_max  H2drained_max  c2_max  end  nwg")
    print("  ".join(f"{x:6.2f}" for x in r))


if __name__ == "__main__":
    main()
