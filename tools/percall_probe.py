"""Host time of each train() call in back-to-back 20-step runs (GPU box diagnostic): modes
plain | nogc | sleepMS | spinMS (an idle / busy gap of MS milliseconds before each run) | psync /
tsync (only the learner-stream sync / only the device sync before each run)."""
import os, sys, time, gc
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import torch
torch.cuda.set_device(0)
from td3_amd.TD3_featured import TD3
from td3_amd.my_replay_buffer import ReplayBuffer_featured as RB
class Box:
    def __init__(self, s): self.shape = tuple(s)
pol = TD3(Box((17,)), Box((6,)), max_action=1.0, device=0, seed=17)
rb = RB(Box((17,)), Box((6,)), max_size=1_000_000, device=0, seed=101)
rb.fill_synthetic(1_000_000, 1.0, seed=7)
for _ in range(5):
    pol.train(rb, 256)
mode = sys.argv[1]
if mode == "nogc":
    gc.collect(); gc.disable()
for rep in range(8):
    if mode != "tsync":
        pol.sync()
    if mode != "psync":
        torch.cuda.synchronize()
    if mode.startswith("sleep"):
        time.sleep(float(mode[5:] or 2) * 1e-3)
    elif mode.startswith("spin"):
        e = time.perf_counter() + float(mode[4:] or 2) * 1e-3
        while time.perf_counter() < e:
            pass
    ts = []
    t0 = time.perf_counter()
    for i in range(20):
        a = time.perf_counter()
        pol.train(rb, 256)
        ts.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    pol.sync(); torch.cuda.synchronize()
    t2 = time.perf_counter()
    if rep < 2 or rep == 7: print(f"{mode} run {rep}: total {1e6*(t2-t0):7.1f} enqueue {1e6*(t1-t0):7.1f} calls " + " ".join(f"{1e6*x:.0f}" for x in ts), flush=True)
