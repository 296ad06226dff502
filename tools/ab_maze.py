"""A/B timing of engine library builds on MazeNavigation (BASELINE config 2:
16x16, 1024 envs, the lane-group kernel), each in its own subprocess:
reset, staggered start phases, 300 untimed steps, then 5 gw_rollout
fragments of 100 steps with HIP events around each launch.

  python tools/ab_maze.py <lib.so> [<lib.so> ...]"""
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
from abmarl_amd.examples.workloads import maze_sim
cc = maze_sim().compiled()
E, H, F = 1024, 200, 100
eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
eng.reset(); eng.all_done.zero_()
eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
acts = torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
out = eng.rollout_buffers(F)
t = 0
ms = []
for f in range(8):
    for s in range(F):
        eng.random_actions(3, t + s, out=acts[s])
    t += F
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); eng.rollout(acts, horizon=H, skip_done_obs=True, out=out); b.record()
    torch.cuda.synchronize()
    if f >= 3:
        ms.append(a.elapsed_time(b))
print(json.dumps({'lib': %(lib)r, 'kernel': eng.kernel, 'launch_ms': ms, 'mean_ms': float(np.mean(ms))}))
'''


def main():
    for lib in sys.argv[1:]:
        code = CHILD % dict(root=ROOT, lib=os.path.abspath(lib))
        r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300)
        print(r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f'{lib}: FAILED {r.stderr[-500:]}',
              flush=True)


if __name__ == '__main__':
    main()
