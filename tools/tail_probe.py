"""Where does a short gw_rollout launch spend its time?  (stamps build)

Runs the bench's TeamBattle setup (4096 envs, staggered phases, pre-roll in
100-step fragments), then one timed fragment of --frag steps, and reads the
per-wave launch stamps (gw_engine.hip STAMP_WAVE: s_memrealtime at the
wave's start / end, HW_ID, XCC_ID).  Prints the launch span, the spread of
wave start times and durations, per-SIMD load (sum of its waves' durations,
the wave count it held) and how durations correlate with the env's work
(acting agent-steps, resets inside the fragment).

  GW_ENGINE_VARIANT=stamps python tools/tail_probe.py [--frag 20] [--envs 4096]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('GW_ENGINE_VARIANT', 'stamps')

from abmarl_amd import _native  # noqa: E402
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim  # noqa: E402

RT_HZ = 100e6   # s_memrealtime


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frag', type=int, default=20)
    ap.add_argument('--envs', type=int, default=4096)
    ap.add_argument('--preroll', type=int, default=1000)
    ap.add_argument('--horizon', type=int, default=200)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    assert _native.VARIANT == 'stamps'
    E, H = args.envs, args.horizon
    eng = GridWorldEngine(team_battle_sim().compiled(), E, seeds=env_seeds(E))
    eng.reset()
    eng.all_done.zero_()
    eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
    F0 = 100
    acts = torch.empty((max(F0, args.frag),) + tuple(eng.actions.shape), dtype=torch.int32,
                       device=eng.device)
    out = eng.rollout_buffers(acts.shape[0])
    t = 0
    while t < args.preroll:
        for s in range(F0):
            eng.random_actions(7, t + s, out=acts[s])
        eng.rollout(acts[:F0], horizon=H, skip_done_obs=True, out=out)
        t += F0
    for rep in range(args.reps):
        for s in range(args.frag):
            eng.random_actions(7, t + s, out=acts[s])
        t += args.frag
        st0 = eng.get_state()
        a0 = eng.acting.clone()
        eng.stamps.zero_()
        torch.cuda.synchronize()
        eng.rollout(acts[:args.frag], horizon=H, skip_done_obs=True, out=out)
        torch.cuda.synchronize()
        st = eng.stamps.cpu().numpy()
        acting = (eng.acting - a0).cpu().numpy().astype(np.int64)
        steps0 = st0['steps'].cpu().numpy() if torch.is_tensor(st0['steps']) else np.asarray(st0['steps'])
        start, end = st[:, 60], st[:, 61]
        hw, xcc = st[:, 62].astype(np.uint64), st[:, 63].astype(np.uint64)
        dur = (end - start) / RT_HZ * 1e6
        span = (end.max() - start.min()) / RT_HZ * 1e6
        wave_id = hw & 0xF
        simd = (hw >> 4) & 0x3
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        x = xcc & 0xF
        print(f'--- rep {rep}: fragment {args.frag} steps, {E} envs')
        print(f'launch span {span:.1f} us; wave starts spread {(start.max() - start.min()) / RT_HZ * 1e6:.1f} us; '
              f'durations median {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} '
              f'p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f} us')
        resets = ((steps0 + args.frag) >= H)  # hit the horizon inside the fragment (lower bound)
        for name, m in [('env reached horizon in fragment', resets), ('no horizon reset', ~resets)]:
            if m.any():
                print(f'  {name:32s}: {m.sum():5d} envs, duration median {np.median(dur[m]):.1f} '
                      f'max {dur[m].max():.1f} us, acting/step median {np.median(acting[m]) / args.frag:.1f}')
        # per SIMD: (xcc, se, sh, cu, simd)
        key = (((x * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
        uk, inv = np.unique(key, return_inverse=True)
        nw = np.bincount(inv)
        load = np.bincount(inv, weights=dur)
        last = np.zeros(len(uk)); np.maximum.at(last, inv, (end - start.min()) / RT_HZ * 1e6)
        print(f'  SIMDs used {len(uk)}, waves per SIMD: {np.bincount(nw).tolist()} (index = count)')
        print(f'  per-SIMD sum of wave durations: median {np.median(load):.0f} max {load.max():.0f} us; '
              f'per-SIMD last end: median {np.median(last):.1f} max {last.max():.1f} us')
        cu_key = key // 4
        ucu, cinv = np.unique(cu_key, return_inverse=True)
        print(f'  CUs used {len(ucu)}, waves per CU: {np.bincount(np.bincount(cinv)).tolist()}')
        c = np.corrcoef(dur, acting)[0, 1]
        print(f'  corr(duration, acting agent-steps) {c:.2f}; acting/env over fragment: median '
              f'{np.median(acting)} max {acting.max()}')
        # the fragment's last step, per phase (s_memtime ticks; stamp 50 = loop top)
        seq = [(50, 10, 'action loads + ballot'), (10, 1, 'tables'), (1, 7, 'attack precheck'),
               (7, 2, 'attack loop'), (2, 11, 'move isolation'), (11, 3, 'serial moves + table'),
               (3, 5, 'observation'), (5, 6, 'dones + state store')]
        ok = (st[:, 50] != 0) & (st[:, 10] > st[:, 50]) & (st[:, 6] > st[:, 10])
        for a, b, nm in seq:
            d = (st[ok, b] - st[ok, a]).astype(np.int64)
            d = d[d > 0]
            if len(d):
                print(f'    last step {nm:24s}: median {np.median(d):7.0f} p90 {np.percentile(d, 90):7.0f} ticks')
        order = np.argsort(-dur)[:8]
        for i in order:
            print(f'    env {i:5d}: {dur[i]:7.1f} us, start +{(start[i] - start.min()) / RT_HZ * 1e6:6.1f}, '
                  f'acting {acting[i]}, steps0 {steps0[i]}, xcc {x[i]} se {se[i]} cu {cu[i]} simd {simd[i]} '
                  f'wave {wave_id[i]}')
        # block -> CU placement: which env ids share a CU, and their SIMDs
        if rep == 0:
            for j in range(2):
                m = np.nonzero(cinv == j)[0]
                print(f'  CU #{j} holds envs {m[:16].tolist()} on SIMDs {simd[m][:16].tolist()} '
                      f'(wave ids {wave_id[m][:16].tolist()})')
        # horizon resets per SIMD: a SIMD with several heavy envs ends last
        hz = np.bincount(inv, weights=resets.astype(np.float64)).astype(int)
        print(f'  SIMDs by envs reaching the horizon in the fragment: {np.bincount(hz).tolist()} (index = count); '
              f'last end by that count: ' + ', '.join(f'{c}: {np.median(last[hz == c]):.1f}'
                                                      for c in range(hz.max() + 1) if (hz == c).any()))


if __name__ == '__main__':
    main()
