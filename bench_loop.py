#!/usr/bin/env python3
"""Environment-steps/s of the full acting + training loop.

    python bench_loop.py [--steps K] [--env-cost-us C] [--config halfcheetah|humanoid]

Runs ``td3_amd.loop.TrainLoop`` (the order of main.py:240-289: act -> env.step -> add -> train,
one train(256) per env step) on a ``SyntheticEnv`` with the config's shapes and a busy-wait of
``--env-cost-us`` per step standing in for the simulator, twice:

* ``overlap``: the build as shipped: train only enqueues its graph; select_action waits only for
  the last actor update, so it overlaps critic-only steps;
* ``serial``: the same loop with a device sync after every train (what a synchronous acting path
  does: the reference's select_action ends in ``.cpu()`` on the training stream).

Prints one JSON line.  Not the BASELINE metric (that is bench.py's gradient-steps/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SHAPES = {"halfcheetah": (17, 6, 1.0), "humanoid": (376, 17, 0.4)}


class _SerialPolicy:
    """The learner with a device sync after every train step (no host/GPU overlap)."""

    def __init__(self, pol):
        self._pol = pol

    def select_action(self, s):
        return self._pol.select_action(s)

    def train(self, rb, b):
        self._pol.train(rb, b)
        self._pol.sync()

    def sync(self):
        self._pol.sync()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(SHAPES), default="halfcheetah")
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--env-cost-us", type=float, default=50.0)
    ap.add_argument("--use-graph", type=int, choices=(0, 1, 2), default=2,
                    help="td3_config.use_graph: 0 direct launches, 1 graph replays, 2 auto (default)")
    args = ap.parse_args()
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    from td3_amd.loop import SyntheticEnv, TrainLoop

    sd, ad, ma = SHAPES[args.config]
    out = {}
    for mode in ("overlap", "serial"):
        np.random.seed(0)
        env = SyntheticEnv(sd, ad, max_action=ma, max_episode_steps=1000, step_cost_us=args.env_cost_us)
        pol = TD3(env.observation_space, env.action_space, max_action=ma, norm="layer",
                  use_graph={0: False, 1: True, 2: "auto"}[args.use_graph])
        rb = ReplayBuffer_featured(env.observation_space, env.action_space, max_size=1_000_000)
        rb.fill_synthetic(100_000, max_action=ma, seed=1)
        p = pol if mode == "overlap" else _SerialPolicy(pol)
        loop = TrainLoop(env, p, rb, max_action=ma, start_policy=0, start_training=0,
                         batch_size=args.batch, expl_noise=0.1)
        loop.run(args.warmup)
        r = loop.run(args.steps)
        out[mode] = r["env_steps_per_s"]
        del pol, rb
    # the same loop without the learner: the host's own ceiling (env + noise + add)
    env = SyntheticEnv(sd, ad, max_action=ma, step_cost_us=args.env_cost_us)
    t0 = time.perf_counter()
    s = env.reset()
    for _ in range(args.steps):
        s, _, d, _ = env.step(np.zeros(ad))
        if d:
            s = env.reset()
    host_only = args.steps / (time.perf_counter() - t0)
    print(json.dumps({
        "metric": f"env-steps/s of the act->env.step->add->train(B={args.batch}) loop, {args.config} shapes",
        "value": round(out["overlap"], 1), "unit": "env-steps/s", "higher_is_better": True,
        "serial_value": round(out["serial"], 1), "speedup_vs_serial": round(out["overlap"] / out["serial"], 3),
        "env_only_steps_per_s": round(host_only, 1), "env_cost_us": args.env_cost_us,
        "steps": args.steps, "warmup": args.warmup, "n_gpus": 1, "use_graph": args.use_graph,
        "data": "SyntheticEnv (tanh linear dynamics + busy-wait per step), replay ring pre-filled with 1e5 "
                "synthetic rows, one train per env step"}))


if __name__ == "__main__":
    main()
