"""Per-phase shader-clock ticks of pac_kernel's turn rollout (BASELINE config 5,
Pacman, 16384 envs, TurnBasedManager), from the stamps build: each wave sums
its turns' ticks per phase (gw_pacman.inc, stamps [30..35]); printed per env
(median / p90 / max) and per turn.

  GW_ENGINE_VARIANT=stamps python tools/stamps_pac.py [envs] [turns]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('GW_ENGINE_VARIANT', 'stamps')

from abmarl_amd import _native  # noqa: E402
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import pacman_sim  # noqa: E402

PHASES = ['reset', 'prologue + actions', 'program (move, overlaps)', 'crowded cells', 'observation',
          'outputs']


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    assert _native.VARIANT == 'stamps'
    H = 200
    eng = GridWorldEngine(pacman_sim().compiled(), E, seeds=env_seeds(E))
    eng.turn_reset()
    eng.all_done.zero_()
    eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
    key = 0x5eed0001
    acts = torch.empty((F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
    out = eng.turn_rollout_buffers(F)
    for rep in range(4):
        for t in range(F):
            eng.random_actions(key, rep * F + t, out=acts[t])
        eng.stamps.zero_()
        eng.turn_rollout(acts, horizon=H, out=out)
    torch.cuda.synchronize()
    st = eng.stamps.cpu().numpy()[:, 30:36].astype(np.float64)
    tot = st.sum(axis=1)
    print(f'pac_kernel turn rollout, {E} envs, {F} turns per launch: ticks per env (whole launch)')
    for k, nm in enumerate(PHASES):
        d = st[:, k]
        print(f'{nm:>26}: median {np.median(d):9.0f} p90 {np.percentile(d, 90):9.0f} max {d.max():9.0f}'
              f'  per turn {np.median(d) / F:7.0f}  share {d.sum() / tot.sum():.3f}')
    print(f'{"total":>26}: median {np.median(tot):9.0f} p90 {np.percentile(tot, 90):9.0f} max {tot.max():9.0f}'
          f'  per turn {np.median(tot) / F:7.0f}')


if __name__ == '__main__':
    main()
