#!/usr/bin/env python3
"""Per-workgroup timeline of the split-K dW launches of one featured step (GPU box helper, not
product code).  Needs the TD3_TL experiment build:

    tools/build_exp.sh tl "-DTD3_TL"
    TD3_LIB=tools/exp/libtd3hip_tl.so python3 tools/tl_dwsk.py   [TL_SHAPE=376,17,1024]

For each dwsk stage: span, entry skew, per-workgroup duration percentiles, and a least-squares
fit dur ~ a * matrix_steps + b * vector_steps + c * segments (us)."""
import ctypes as C
import os
import sys

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
    lib.td3_tl_read.restype = C.c_int
    lib.td3_tl_read.argtypes = [C.c_void_p, C.c_int]
    lib.td3_tl_clear.restype = C.c_int
    sd, ad, B = (int(x) for x in os.environ.get("TL_SHAPE", "376,17,1024").split(","))
    pol = TD3(Box((sd,)), Box((ad,)), max_action=0.4, norm="layer", device=0, seed=17, use_graph=False)
    rb = RB(Box((sd,)), Box((ad,)), max_size=20_000, device=0, seed=3)
    rb.fill_synthetic(rb.max_size, 0.4, seed=7)
    for _ in range(10):
        pol.train(rb, B)
    pol.sync()
    h = pol._h
    ms = (C.c_float * 128)()
    n = C.c_int()
    buf = np.zeros((8192, 8), dtype=np.uint64)
    for phase in (0, 1):
        _lib.check(lib.td3_profile_stages(h, rb.handle, B, phase, ms, 128, C.byref(n)), "profile")
        for i in range(1, n.value):
            kern = lib.td3_stage_kernel(h, i).decode()
            if "dwsk" not in kern:
                continue
            name = lib.td3_stage_name(h, i).decode()
            t = C.c_float()
            _lib.check(lib.td3_time_stage(h, i, 20, C.byref(t)), "time")
            lib.td3_tl_clear()
            _lib.check(lib.td3_time_stage(h, i, 1, C.byref(t)), "time1")
            lib.td3_tl_read(buf.ctypes.data, 8192)
            v = buf[(buf[:, 3] != 0)].astype(np.int64)
            base = v[:, 0].min()
            dur = (v[:, 3] - v[:, 0]) * 0.01
            end = (v[:, 3] - base) * 0.01
            mat, vec, seg = v[:, 5], v[:, 6], v[:, 7]
            print(f"== phase {phase} {name} {kern}: stage {t.value * 1e3:6.2f} us (20-run avg), wgs {len(v)}, "
                  f"span {end.max():6.2f}, entry skew {(v[:, 0].max() - base) * 0.01:5.2f}")
            print("   dur p10/50/90/max", np.round(np.percentile(dur, [10, 50, 90, 100]), 2).tolist(),
                  " end p50/90/max", np.round(np.percentile(end, [50, 90, 100]), 2).tolist())
            A = np.stack([mat, vec, seg], 1).astype(np.float64)
            coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
            print(f"   fit: {coef[0]:.3f} us/matrix step, {coef[1]:.3f} us/vector step, {coef[2]:.3f} us/segment;"
                  f" resid p90 {np.percentile(np.abs(A @ coef - dur), 90):.2f}")
            first = (v[:, 1] - v[:, 0]) * 0.01
            print(f"   steps per wg: matrix p50/max {np.median(mat):.0f}/{mat.max()}, vector p50/max "
                  f"{np.median(vec):.0f}/{vec.max()}, segments p50/max {np.median(seg):.0f}/{seg.max()};"
                  f" first segment p50 {np.median(first):.2f}")
            slow = np.argsort(-end)[:6]
            for j in slow:
                print(f"   late wg: end {end[j]:6.2f} entry {(v[j, 0] - base) * 0.01:5.2f} dur {dur[j]:6.2f} "
                      f"mat {mat[j]} vec {vec[j]} seg {seg[j]} xcc {v[j, 4] & 0xFFFF}")


if __name__ == "__main__":
    main()
