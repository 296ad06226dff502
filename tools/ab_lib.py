"""A/B timing of engine library builds on the same GPU box (tools only).

  python tools/ab_lib.py <lib.so> [<lib.so> ...]

Each library runs in its own subprocess: TeamBattle 32x32 / 64 agents /
4096 envs, reset, start phases staggered over the horizon, 600 untimed
steps, then 300 steps with HIP events around the step kernel; prints
ms/step and the event-timed step kernel average per library."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes as C, json, sys, time
sys.path.insert(0, %(root)r)
import numpy as np, torch
REPS = int(%(reps)r)
from abmarl_amd import _native
_native.LIB = %(lib)r
sigs = dict(_native.SIGNATURES)
L = C.CDLL(_native.LIB)
for n in list(sigs):
    if not hasattr(L, n):
        del _native.SIGNATURES[n]
from abmarl_amd.engine import GridWorldEngine, env_seeds
from abmarl_amd.examples.workloads import team_battle_sim
cc = team_battle_sim().compiled()
E, H = 4096, 200
eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
eng.reset(); eng.all_done.zero_()
st = eng.get_state()
eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
for t in range(600):
    eng.random_actions(7, t); eng.step_autoreset_next(horizon=H)
torch.cuda.synchronize()
K = 300
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
a0 = int(eng.acting.sum().item())
t0 = time.perf_counter()
for t in range(K):
    eng.random_actions(7, 600 + t)
    evs[t][0].record(); eng.step_autoreset_next(horizon=H); evs[t][1].record()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
res = {'lib': %(lib)r, 'ms_per_step': dt / K * 1e3,
       'kernel_ms': float(np.mean([a.elapsed_time(b) for a, b in evs])),
       'agent_steps_per_s': (int(eng.acting.sum().item()) - a0) / dt}
if hasattr(L, 'gw_rollout'):
    # the same steps continued as fragments of F steps, one launch each
    for F in (20, 100):
        acts = torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
        out = eng.rollout_buffers(F)
        rates = []
        for rep in range(REPS):
            for s in range(F):
                eng.random_actions(9, 100000 + rep * F + s, out=acts[s])
            torch.cuda.synchronize()
            a0 = int(eng.acting.sum().item())
            t0 = time.perf_counter()
            eng.rollout(acts, horizon=H, skip_done_obs=True, out=out)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            rates.append(((int(eng.acting.sum().item()) - a0) / dt, dt / F * 1e3))
        rates.sort()
        res[f'rollout{F}_skip'] = {'agent_steps_per_s_median': rates[len(rates) // 2][0],
                                   'ms_per_step_median': sorted(r[1] for r in rates)[len(rates) // 2],
                                   'agent_steps_per_s_best': rates[-1][0]}
print(json.dumps(res))
'''

for lib in sys.argv[1:]:
    out = subprocess.run([sys.executable, '-c', CHILD % dict(root=ROOT, lib=os.path.abspath(lib), reps=os.environ.get('AB_REPS', '7'))],
                         capture_output=True, text=True, timeout=300)
    line = [x for x in out.stdout.splitlines() if x.startswith('{')]
    print(line[-1] if line else json.dumps({'lib': lib, 'error': out.stderr[-800:]}), flush=True)
