"""Probe: host/launch overhead of the TeamBattle rollout step on the GPU.

Times K steps of random actions + NEXT_STEP step four ways:
  events  two C-ABI calls per step, HIP events around the step kernel
  lean    one gw_rollout_step call per step, no events
  graph   K gw_rollout_step calls captured in one HIP graph, replayed once
  graph+events  the same with timing events captured around each step
and prints ms/step for each (and the event-timed step kernel average)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim  # noqa: E402

K, PRE = 200, 600
cc = team_battle_sim().compiled()
out = {}


def fresh():
    eng = GridWorldEngine(cc, 4096, seeds=env_seeds(4096))
    eng.reset()
    eng.all_done.zero_()
    for t in range(PRE):
        eng.rollout_step(7, t, horizon=200)
    torch.cuda.synchronize()
    return eng


eng = fresh()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(K):
    eng.random_actions(7, PRE + t)
    evs[t][0].record()
    eng.step_autoreset_next(horizon=200)
    evs[t][1].record()
torch.cuda.synchronize()
out['events_ms_per_step'] = (time.perf_counter() - t0) / K * 1e3
out['events_kernel_ms'] = sum(a.elapsed_time(b) for a, b in evs) / K

eng = fresh()
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in range(K):
    eng.rollout_step(7, PRE + t, horizon=200)
torch.cuda.synchronize()
out['lean_ms_per_step'] = (time.perf_counter() - t0) / K * 1e3

eng = fresh()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.graph(g, stream=s):
    for t in range(K):
        eng.rollout_step(7, PRE + t, horizon=200)
torch.cuda.synchronize()
t0 = time.perf_counter()
g.replay()
torch.cuda.synchronize()
out['graph_ms_per_step'] = (time.perf_counter() - t0) / K * 1e3

try:
    eng = fresh()
    g2 = torch.cuda.CUDAGraph()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g2, stream=s):
        for t in range(K):
            eng.random_actions(7, PRE + t)
            evs[t][0].record()
            eng.step_autoreset_next(horizon=200)
            evs[t][1].record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g2.replay()
    torch.cuda.synchronize()
    out['graph_events_ms_per_step'] = (time.perf_counter() - t0) / K * 1e3
    out['graph_events_kernel_ms'] = sum(a.elapsed_time(b) for a, b in evs) / K
except Exception as ex:  # noqa: BLE001
    out['graph_events_error'] = repr(ex)[:300]
print(json.dumps(out))
