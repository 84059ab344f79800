#!/usr/bin/env python3
"""Data-parallel step cost on ONE GPU (GPU box helper, not product code): a 1-rank RCCL
communicator attached to the learner, so every step runs the DP stage list (grad-only dW ->
ncclAllReduce -> flat Adam / Polyak).  Times the plain step, the DP step with direct launches
(use_graph auto) and the DP step replayed from a captured hipGraph (RCCL captured).

    python3 tools/dp1_probe.py [steps]
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def run(mode, steps):
    import torch
    from td3_amd import _lib
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured as RB
    use_graph = {"plain": "auto", "dp_auto": "auto", "dp_graph": True, "dp_eager": False}[mode]
    torch.manual_seed(1000)
    pol = TD3(Box((17,)), Box((6,)), max_action=1.0, norm="layer", device=0, seed=17, use_graph=use_graph)
    rb = RB(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=101)
    rb.fill_synthetic(1_000_000, 1.0, seed=7)
    if mode != "plain":
        uid = (C.c_ubyte * 128)()
        _lib.check(pol._lib.td3_comm_unique_id(uid), "uid")
        _lib.check(pol._lib.td3_comm_init(pol._h, uid, 1, 0), "comm_init")
    for _ in range(50):
        pol.train(rb, 256)
    pol.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        pol.train(rb, 256)
    t_host = time.perf_counter() - t0
    pol.sync()
    dt = time.perf_counter() - t0
    print(f"{mode:10s} {steps / dt:9.1f} steps/s  {dt / steps * 1e6:7.1f} us/step  "
          f"(host enqueue {t_host / steps * 1e6:6.1f} us/step)", flush=True)
    return pol


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    import torch
    torch.cuda.set_device(0)
    for mode in ("plain", "dp_auto", "dp_eager", "dp_graph"):
        run(mode, steps)


if __name__ == "__main__":
    main()
