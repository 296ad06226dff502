"""Why is a single timed 20-step gw_rollout launch slower than the mean of
back-to-back ones?  Times one 20-step fragment (HIP events) after:
  a) back-to-back with the previous launch (no host sync between),
  b) a host sync + a short idle (sleep_ms) before it,
  c) as b) on a freshly allocated action buffer (written just before).
TeamBattle 32x32, 64 agents, 4096 envs, 1000-step pre-roll as bench.py.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim  # noqa: E402

E, F, H = 4096, 20, 200
sim = team_battle_sim()
cc = sim.compiled()
eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
eng.reset()
eng.all_done.zero_()
eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
acts = torch.empty((100,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
out = eng.rollout_buffers(100)
t = 0
for _ in range(10):
    for s in range(100):
        eng.random_actions(7, t + s, out=acts[s])
    eng.rollout(acts, horizon=H, skip_done_obs=True, out=out)
    t += 100
torch.cuda.synchronize()


def timed(buf, n=1):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        eng.rollout(buf[:F], horizon=H, skip_done_obs=True, out=out)
        b.record()
    torch.cuda.synchronize()
    return [round(a.elapsed_time(b), 4) for a, b in evs]


res = {}
res['back_to_back_x8'] = timed(acts, 8)
for sleep_ms in (0, 1, 10, 100):
    torch.cuda.synchronize()
    time.sleep(sleep_ms / 1e3)
    res[f'after_sync_sleep_{sleep_ms}ms'] = timed(acts, 2)
fresh = torch.empty_like(acts[:F])
for s in range(F):
    eng.random_actions(9, s, out=fresh[s])
torch.cuda.synchronize()
res['fresh_buffer'] = timed(fresh, 2)
# a busy GPU right up to the launch (a 100-step fragment queued before it)
eng.rollout(acts, horizon=H, skip_done_obs=True, out=out)
res['after_busy_queue'] = timed(acts, 1)
print(json.dumps(res))
