"""Where the time of one short gw_rollout fragment goes (bench.py's default
driver window is ONE 20-step launch): host time of the call, HIP-event time
around it, and the same with the launch already queued behind a spin kernel
(so the host launch latency is hidden and the events see the kernel alone).

usage: python tools/launch_probe.py [--envs 4096] [--frag 20] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from abmarl_amd.engine import GridWorldEngine, env_seeds      # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=4096)
    ap.add_argument('--frag', type=int, default=20)
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    E, F = a.envs, a.frag
    eng = GridWorldEngine(team_battle_sim().compiled(), E, seeds=env_seeds(E))
    eng.reset()
    eng.all_done.zero_()
    eng.set_state(steps=torch.as_tensor((np.arange(E) * 200 // E).astype(np.int32), device=eng.device))
    acts = torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
    out = eng.rollout_buffers(F)
    t = 0

    def fill():
        nonlocal t
        for s in range(F):
            eng.random_actions(7, t + s, out=acts[s])
        t += F

    for _ in range(20):                      # pre-roll: steady state
        fill()
        eng.rollout(acts, horizon=200, skip_done_obs=True, out=out)
    torch.cuda.synchronize()
    res = {'host_call_us': [], 'event_us': [], 'wall_us': [], 'event_queued_us': []}
    for _ in range(a.reps):
        fill()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        e0.record()
        h0 = time.perf_counter()
        eng.rollout(acts, horizon=200, skip_done_obs=True, out=out)
        h1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        w1 = time.perf_counter()
        res['host_call_us'].append((h1 - h0) * 1e6)
        res['event_us'].append(e0.elapsed_time(e1) * 1e3)
        res['wall_us'].append((w1 - w0) * 1e6)
        # queued: a sleep kernel first, so the rollout launch is enqueued
        # before the GPU reaches it (events then bracket the kernel alone)
        fill()
        torch.cuda.synchronize()
        torch.cuda._sleep(2_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.rollout(acts, horizon=200, skip_done_obs=True, out=out)
        e1.record()
        torch.cuda.synchronize()
        res['event_queued_us'].append(e0.elapsed_time(e1) * 1e3)
    print(json.dumps({k: [round(float(np.median(v)), 1), round(float(np.min(v)), 1), round(float(np.max(v)), 1)]
                      for k, v in res.items()} | {'envs': E, 'frag': F, 'stat': 'median, min, max'}))


if __name__ == '__main__':
    main()
