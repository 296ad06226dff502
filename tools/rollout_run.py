"""A short TeamBattle rollout for rocprofv3 (kernel trace / PMC passes):
4096 envs, start phases staggered over the horizon, 200 untimed single
steps, then `--frags` fragments of `--frag` steps through gw_rollout.

  python tools/rollout_run.py [--frag 100] [--frags 3] [--skip]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--frag', type=int, default=100)
ap.add_argument('--frags', type=int, default=3)
ap.add_argument('--envs', type=int, default=4096)
ap.add_argument('--skip', action='store_true')
args = ap.parse_args()
E, H = args.envs, 200
eng = GridWorldEngine(team_battle_sim().compiled(), E, seeds=env_seeds(E))
eng.reset()
eng.all_done.zero_()
eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
for t in range(200):
    eng.rollout_step(3, t, horizon=H)
acts = torch.empty((args.frag,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
out = eng.rollout_buffers(args.frag)
for f in range(args.frags):
    for s in range(args.frag):
        eng.random_actions(3, 200 + f * args.frag + s, out=acts[s])
    torch.cuda.synchronize()
    a0 = int(eng.acting.sum().item())
    t0 = time.perf_counter()
    eng.rollout(acts, horizon=H, skip_done_obs=args.skip, out=out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f'fragment {f}: {args.frag} steps, {dt / args.frag * 1e3:.4f} ms/step, '
          f'{(int(eng.acting.sum().item()) - a0) / dt / 1e9:.3f} G agent-steps/s', flush=True)
