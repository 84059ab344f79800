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


def _gate(torch):
    """A host-written word the learner stream waits on (hipStreamWaitValue32): the steps are queued
    behind it while the GPU idles, then released at once, so the span has no host starvation."""
    hip = C.CDLL("libamdhip64.so")
    hip.hipStreamWaitValue32.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint, C.c_uint32]
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    return hip, word


def _set_flags(when):
    """SP_SPIN=pre|post[:flag]: hipSetDeviceFlags(flag) (1 spin, 2 yield, 4 blocking sync) before
    the first HIP call or after torch made the device current."""
    spec = os.environ.get("SP_SPIN", "")
    if not spec.startswith(when):
        return
    flag = int(spec.split(":")[1]) if ":" in spec else 1
    hip = C.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(C.c_uint(flag))
    print(f"hipSetDeviceFlags({flag}) {when} -> {rc}", flush=True)


def main():
    _set_flags("pre")
    import torch
    torch.cuda.set_device(0)
    _set_flags("post")
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured as RB
    steps = int(os.environ.get("SP_STEPS", "20"))
    mode = os.environ.get("SP_MODE", "plain")          # plain | gate | sleep | syncs
    ug = {"auto": "auto", "1": True, "0": False}[os.environ.get("SP_GRAPH", "auto")]
    pol = TD3(Box((17,)), Box((6,)), max_action=1.0, device=0, seed=17, use_graph=ug)
    rb = RB(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=101)
    rb.fill_synthetic(1_000_000, 1.0, seed=7)
    for _ in range(5):
        pol.train(rb, 256)
    sp = int(pol._lib.td3_stream(pol._h))
    stream = torch.cuda.ExternalStream(sp, device=0)
    hip, word = _gate(torch) if mode == "gate" else (None, None)
    per_call = [[], []]
    if mode == "syncs":                                # what each way of ending a timed run costs
        import numpy as np
        forms = {"td3_sync + torch sync": lambda: (pol.sync(), torch.cuda.synchronize()),
                 "torch sync only": lambda: torch.cuda.synchronize(),
                 "td3_sync only": lambda: pol.sync(),
                 "td3_sync + stream sync + torch sync": lambda: (pol.sync(), stream.synchronize(),
                                                                 torch.cuda.synchronize()),
                 "stream sync + torch sync": lambda: (stream.synchronize(), torch.cuda.synchronize())}
        for name, fn in forms.items():
            tt = []
            for rep in range(12):
                pol.sync()
                torch.cuda.synchronize()
                for i in range(steps):
                    pol.train(rb, 256)
                time.sleep(0.003)                      # the GPU is done: time the ending alone
                a = time.perf_counter()
                fn()
                tt.append(time.perf_counter() - a)
            print(f"syncs: {name:40s} median {1e6 * np.median(tt):6.1f} us  min {1e6 * min(tt):6.1f}", flush=True)
        return
    for rep in range(8):
        pol.sync()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode == "gate":
            word[0] = 0
            assert hip.hipStreamWaitValue32(sp, word.data_ptr(), 1, 0, 0xFFFFFFFF) == 0
        elif mode == "sleep":
            with torch.cuda.stream(stream):
                torch.cuda._sleep(20_000_000)
        t0 = time.perf_counter()
        e0.record(stream)
        t1 = time.perf_counter()
        for i in range(steps):
            a = time.perf_counter()
            pol.train(rb, 256)
            per_call[i % 2].append(time.perf_counter() - a)
        t2 = time.perf_counter()
        e1.record(stream)
        if mode == "gate":
            word[0] = 1
        pol.sync()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        gpu = e0.elapsed_time(e1) * 1e3
        print(f"{mode}/{os.environ.get('SP_GRAPH', 'auto')} run {rep}: host {1e6 * (t4 - t0):7.1f} us (enqueue {1e6 * (t2 - t1):6.1f}, "
              f"sync {1e6 * (t3 - t2):6.1f}, torch sync {1e6 * (t4 - t3):5.1f})  gpu events {gpu:7.1f} us = "
              f"{gpu / steps:6.2f} us/step", flush=True)
    import numpy as np
    print(f"{mode}: host per train() call: first-of-pair median {1e6 * np.median(per_call[0]):.1f} us, "
          f"second {1e6 * np.median(per_call[1]):.1f} us", flush=True)


if __name__ == "__main__":
    main()
