"""bench.py's timed-region pattern, repeated: a fresh action buffer for the
20 timed steps (torch.empty), random_actions into it, sync + .item(), then
ONE 20-step gw_rollout launch timed with HIP events.  Variants: (a) fresh
buffer every rep, (b) the same buffer reused, (c) fresh buffer with an
untimed read pass over it first (a 1-step rollout on slab 0)."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim  # noqa: E402

E, F, H = 4096, 20, 200
cc = team_battle_sim().compiled()
eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
eng.reset(); eng.all_done.zero_()
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
res = {k: [] for k in ('fresh', 'reused', 'fresh_touched', 'wall_fresh_ms')}
keep = torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
for rep in range(4):
    for kind in ('fresh', 'reused', 'fresh_touched'):
        buf = keep if kind == 'reused' else torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32,
                                                        device=eng.device)
        for s in range(F):
            eng.random_actions(9, t + s, out=buf[s])
        if kind == 'fresh_touched':
            eng.rollout(buf[:1], horizon=H, skip_done_obs=True, out=out)
            t += 1
        torch.cuda.synchronize()
        _ = int(eng.acting.sum().item())
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        eng.rollout(buf, horizon=H, skip_done_obs=True, out=out)
        b.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        t += F
        res[kind].append(round(a.elapsed_time(b), 4))
        if kind == 'fresh':
            res['wall_fresh_ms'].append(round(wall, 4))
        del buf
print(json.dumps(res))
