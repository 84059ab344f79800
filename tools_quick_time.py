import time, sys, numpy as np, torch
sys.path.insert(0, '.')
from td3_amd.TD3_featured import TD3
from td3_amd.my_replay_buffer import ReplayBuffer_featured
class Box:
    def __init__(s, shape): s.shape = shape
sd, ad, B = 17, 6, 256
pol = TD3(Box((sd,)), Box((ad,)), max_action=1.0, norm="layer")
rb = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=1000000)
rb.fill_synthetic(1000000, 1.0, 1)
for i in range(20): pol.train(rb, B)
pol.sync()
names = []
ms = (__import__('ctypes').c_float * 64)()
n = __import__('ctypes').c_int()
for ap in (0, 1):
    rc = pol._lib.td3_profile_stages(pol._h, rb.handle, B, ap, ms, 64, __import__('ctypes').byref(n))
    assert rc == 0, pol._lib.td3_last_error()
    tot = 0
    for i in range(n.value):
        print(f"  phase{ap} {pol._lib.td3_stage_name(pol._h, i).decode():16s} {ms[i]*1000:8.1f} us")
        tot += ms[i]
    print(f"phase{ap} total {tot*1000:.1f} us (eager, with event gaps)")
for K in (200, 1000):
    torch.cuda.synchronize(); t = time.perf_counter()
    for i in range(K): pol.train(rb, B)
    pol.sync(); torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"K={K}: {K/dt:.1f} grad-steps/s  {dt/K*1e6:.1f} us/step")
