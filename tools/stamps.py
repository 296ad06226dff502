"""Per-phase s_memtime stamps of the step kernel (GW_ENGINE_VARIANT=stamps
build, -DGW_STAMPS): runs a workload for a few steps and prints, per phase
(consecutive stamp indices), the median / p90 / max over envs of the shader
clock ticks spent, for one plain step launch and one launch that resets.

  GW_ENGINE_VARIANT=stamps python tools/stamps.py [rtt|team_battle] [envs]
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
import bench  # noqa: E402

STEP = {0: 'start', 1: 'prologue+tables', 2: 'attack pass', 3: 'move pass', 4: 'table rebuild',
        5: 'obs windows', 6: 'crowded draws', 7: 'obs store', 8: 'dones', 9: 'store state'}
RESET = {12: 'reset start', 17: 'first state component', 13: 'second state component',
         14: 'tables', 15: 'obs windows', 16: 'crowded draws'}
# inside the parallel placement (ReachTheTarget workgroup kernel)
PLACE = {17: 'placement start', 18: 'removal masks', 19: 'draw offsets', 20: 'Jacobi sweeps'}


def report(st, order, names, title):
    print(f'--- {title}')
    prev = None
    for i in order:
        if prev is not None:
            d = st[:, i] - st[:, prev]
            ok = (st[:, i] != 0) & (st[:, prev] != 0)
            if ok.any():
                d = d[ok]
                print(f'{names.get(i, i):>24}: median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}'
                      f'  max {d.max():9.0f}  ({ok.sum()} envs)')
        prev = i


# one-wave-per-env kernel (gw_engine.hip step_kernel, STAMP indices)
TB_STEP = {0: 'start', 10: 'prologue', 1: 'tables', 7: 'attack precheck', 2: 'attack loop',
           11: 'move isolation', 3: 'serial moves+table', 4: '-',
           8: 'obs windows', 9: 'crowded draws', 5: 'obs store', 6: 'dones+store'}
TB_NEXT = {0: 'start', 10: 'prologue', 12: '-', 11: 'placement', 15: 'health', 13: '-',
           26: 'tables+obs windows', 27: 'crowded draws', 14: 'obs store', 6: 'state store'}


NSTEPS = int(os.environ.get('NSTEPS', '430'))


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else 'rtt'
    E = int(sys.argv[2]) if len(sys.argv) > 2 else (1024 if wl == 'rtt' else 4096)
    assert _native.VARIANT == 'stamps'
    cc = (bench.rtt_sim() if wl == 'rtt' else bench.team_battle_sim()).compiled()
    eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
    eng.stamps.zero_()
    eng.reset()
    torch.cuda.synchronize()
    st = eng.stamps.cpu().numpy()
    report(st, [12, 17, 13, 14, 15, 16], RESET, f'{wl}: reset launch ({E} envs)')
    if wl == 'rtt' and (st[:, 20] != 0).any():
        report(st, [17, 18, 19, 20], PLACE, 'parallel placement')
        sw = st[:, 21]
        print(f'{"sweeps":>24}: median {np.median(sw):.0f} max {sw.max()}')
    eng.all_done.zero_()
    # episode phases spread over the horizon, as in bench.py (steady state:
    # about E/200 envs reset in every launch)
    H = 200
    eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
    for t in range(NSTEPS):
        eng.random_actions(1, t)
        eng.stamps.zero_()
        eng.step_autoreset_next(horizon=H)
    torch.cuda.synchronize()
    st = eng.stamps.cpu().numpy()
    if wl == 'rtt':
        report(st, list(range(10)), STEP, f'{wl}: step launch {NSTEPS} (next_step auto-reset)')
        if (st[:, 35] != 0).any():
            report(st, [5, 30, 31, 32, 35], {30: 'crowd: members ranked', 31: 'crowd: pairs + words',
                                             32: 'crowd: offset scans', 35: 'crowd: values'},
                   'crowded draws, parallel form')
            ok = st[:, 35] != 0
            print(f'{"pairs":>24}: median {np.median(st[ok, 33]):.0f} max {st[ok, 33].max()}; members median '
                  f'{np.median(st[ok, 34]):.0f} max {st[ok, 34].max()}; scan passes median '
                  f'{np.median(st[ok, 36]):.0f} max {st[ok, 36].max()}')
        tot = st[:, 9] - st[:, 0]
    else:
        stepped = st[:, 2] != 0
        report(st[stepped], [0, 10, 1, 7, 2, 11, 3, 4, 8, 9, 5, 6], TB_STEP,
               f'{wl}: step launch {NSTEPS}, stepping envs ({stepped.sum()})')
        if (~stepped).any():
            report(st[~stepped], [0, 10, 12, 11, 15, 13, 26, 27, 14, 6], TB_NEXT,
                   f'{wl}: resetting envs ({(~stepped).sum()})')
        rs = st[~stepped]
        print('health: rng.pos at start', rs[:, 40].tolist(), 'nrand', rs[:, 41].tolist())
        for k, nm in enumerate(['word buffer', 'list lengths', 'draw offsets', 'rank+fixpoint', 'final']):
            print(f'   jacobi {nm:>14}: median {np.median(rs[:, 20 + k]):8.0f} max {rs[:, 20 + k].max():8.0f}')
        print(f'   jacobi sweeps: median {np.median(rs[:, 25]):.0f} max {rs[:, 25].max()}')
        tot = st[:, 6] - st[:, 0]
        print(f'launch span (last end - first start, if the counter is global): '
              f'{st[:, 6].max() - st[:, 0].min()} ticks; starts spread over {st[:, 0].max() - st[:, 0].min()}')
    if wl != 'rtt':
        ns, na = st[:, 28], st[:, 29]
        at = st[:, 2] - st[:, 1]
        ok = ns > 0
        print(f'attackers per env: median {np.median(na):.0f}, with a possible target {np.median(ns):.0f} '
              f'(max {ns.max()}); attack ticks per such attacker: median {np.median(at[ok] / ns[ok]):.0f}')
        print(f'movers per env: median {np.median(st[:, 31]):.0f}, not isolated (serial) median '
              f'{np.median(st[:, 30]):.0f} max {st[:, 30].max()}')
        cnt = st[:, 48]
        if cnt.sum() > 0:
            okc = cnt > 0
            print(f'serial attack_one calls: {int(cnt.sum())} in {okc.sum()} envs; per call (sum over envs / calls), '
                  f'median of per-env means:')
            for k, nm in zip(range(42, 48), ['window scan + ranks', 'accuracy draws', 'subset draws',
                                             'attacked list', 'damage + cell table', 'rewards']):
                per_env = st[okc, k] / cnt[okc]
                print(f'   {nm:>22}: {st[:, k].sum() / cnt.sum():8.0f}   median {np.median(per_env):8.0f}')
            loop = (st[:, 2] - st[:, 7])
            print(f'   {"loop total / call":>22}: {loop[okc].sum() / cnt.sum():8.0f}')
        for lo, hi in [(0, 4), (4, 8), (8, 16), (16, 64)]:
            m = (ns >= lo) & (ns < hi)
            if m.any():
                print(f'   {lo:2d}-{hi:2d} possible-target attackers: {m.sum():5d} envs, attack pass median '
                      f'{np.median(at[m]):.0f} ticks')
    print(f'whole launch per env: median {np.median(tot):.0f} p99 {np.percentile(tot, 99):.0f} '
          f'max {tot.max():.0f} ticks')


if __name__ == '__main__':
    main()
