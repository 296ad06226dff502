"""A/B timing of engine library builds on the headline workload (TeamBattle
32x32, 64 agents, 4096 envs, next_step auto-reset, skip_done_obs), each in
its own subprocess: reset, staggered start phases, a 300-step pre-roll, then
gw_rollout fragments of 20 and of 100 steps with HIP events around each
launch (the mean of the last five of each).

  python tools/ab_headline.py [--envs N] <lib.so> [<lib.so> ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, %(root)r)
import numpy as np, torch
from abmarl_amd import _native
_native.LIB = %(lib)r
from abmarl_amd.engine import GridWorldEngine, env_seeds
from abmarl_amd.examples.workloads import team_battle_sim
cc = team_battle_sim().compiled()
E, H = %(envs)d, 200
eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
eng.reset(); eng.all_done.zero_()
eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
res = {'lib': %(lib)r, 'envs': E, 'kernel': eng.kernel}
t = 0
for F, n in ((100, 3), (20, 8), (100, 8)):
    acts = torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
    out = eng.rollout_buffers(F)
    ms = []
    for f in range(n):
        for s in range(F):
            eng.random_actions(3, t + s, out=acts[s])
        t += F
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); eng.rollout(acts, horizon=H, skip_done_obs=True, out=out); b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    if n == 8:
        res[f'f{F}_ms'] = float(np.mean(ms[-5:]))
        res[f'f{F}_all'] = [round(x, 4) for x in ms]
print(json.dumps(res))
'''


def main():
    args = sys.argv[1:]
    envs = 4096
    if args and args[0] == '--envs':
        envs, args = int(args[1]), args[2:]
    for lib in args:
        code = CHILD % dict(root=ROOT, lib=os.path.abspath(lib), envs=envs)
        r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300)
        print(r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f'{lib}: FAILED {r.stderr[-800:]}',
              flush=True)


if __name__ == '__main__':
    main()
