"""Diagnostic: per-phase cycle shares of step_kernel from s_memtime stamps.

Builds/loads libgw_engine_stamps.so (-DGW_STAMPS), runs the bench workload
and prints the median cycles between consecutive stamps over envs & steps.
Read the SHARES, not the absolute time (stamps serialise the schedule).
usage (GPU): GW_ENGINE_STAMPS=1 python tools/stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ['GW_ENGINE_STAMPS'] = '1'

from abmarl_amd import _native  # noqa: E402
_native.build(stamps=True)
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
import bench  # noqa: E402

NAMES = {0: 'start', 1: 'tables', 10: 'load', 2: 'attack', 3: 'move', 4: 'cells', 8: 'obs-par', 9: 'obs-ev',
         5: 'obs-store', 6: 'dones+store'}


HORIZON = int(os.environ.get('HORIZON', '100000'))
MODE = os.environ.get('MODE', 'same_step')


def main():
    cc = bench.team_battle_sim().compiled()
    E = int(os.environ.get('ENVS', '4096'))
    eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
    L = eng.L
    L.gw_debug_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
    st = torch.zeros((E, 32), dtype=torch.int64, device=eng.device)
    L.gw_debug_set_stamps(eng.h, C.c_void_p(st.data_ptr()))
    eng.reset()
    eng.all_done.zero_()
    order = [0, 10, 1, 2, 3, 4, 8, 9, 5, 6]
    deltas = []
    ends = []
    resets = []
    kms, span, emax = [], [], []
    for t in range(int(os.environ.get('STEPS', '300'))):
        eng.random_actions(7, t)
        st.zero_()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        (eng.step_autoreset_next if MODE == 'next_step' else eng.step_autoreset)(horizon=HORIZON)
        ev1.record()
        torch.cuda.synchronize()
        s = st.cpu().numpy()
        if t >= 20:
            kms.append(ev0.elapsed_time(ev1))
            span.append(int(s[:, 6].max() - s[:, 0].min()))
            emax.append(int((s[:, 6] - s[:, 0]).max()))
        if t >= 20:
            stepped = s[:, 1] != 0
            d = np.stack([s[stepped, order[i + 1]] - s[stepped, order[i]] for i in range(len(order) - 1)], 1)
            deltas.append(d)
            ends.append(s[:, 6] - s[:, 0])
            rs = s[s[:, 12] != 0]
            if len(rs):
                resets.append(np.stack([rs[:, 10] - rs[:, 0], rs[:, 13] - rs[:, 12],
                                        rs[:, 14] - rs[:, 13], rs[:, 6] - rs[:, 0],
                                        rs[:, 11] - rs[:, 12], rs[:, 15] - rs[:, 11],
                                        rs[:, 16], rs[:, 17], rs[:, 18], rs[:, 19],
                                        rs[:, 20], rs[:, 21], rs[:, 22], rs[:, 23], rs[:, 24], rs[:, 25],
                                        rs[:, 26] - rs[:, 13], rs[:, 27] - rs[:, 26], rs[:, 14] - rs[:, 27]], 1))
    d = np.concatenate(deltas)
    tot = d.sum(1)
    print(f"per-env cycles (s_memtime ticks): median {np.median(tot):.0f} p90 "
          f"{np.percentile(tot, 90):.0f} max {tot.max()}")
    for i in range(len(order) - 1):
        print(f"  {NAMES[order[i]]:>8s} -> {NAMES[order[i+1]]:<12s} median {np.median(d[:, i]):8.0f}"
              f"  mean {d[:, i].mean():8.0f}  share {d[:, i].sum() / tot.sum() * 100:5.1f}%")
    print(f"kernel ms (events) mean {np.mean(kms):.4f}; stamp span (last end - first start) mean "
          f"{np.mean(span):.0f} ticks -> {np.mean(span) / np.mean(kms) / 1e6:.3f} ticks/ns; "
          f"max env duration mean {np.mean(emax):.0f} ticks")
    e = np.concatenate(ends)
    print(f"whole env (stamp 0 -> 6): median {np.median(e):.0f} p99 {np.percentile(e, 99):.0f} "
          f"max {e.max()}")
    print(f"load (lanes+rng+actions, 0->10) median {np.median(d[:, 0] * 0 + (np.concatenate(deltas)[:, 0])):.0f}")
    if resets:
        r = np.concatenate(resets)
        print(f"reset envs: {len(r)}; median cycles: load {np.median(r[:, 0]):.0f}, do_reset "
              f"{np.median(r[:, 1]):.0f}, reset tables+obs {np.median(r[:, 2]):.0f}, whole env "
              f"{np.median(r[:, 3]):.0f} (max {r[:, 3].max()}); placement {np.median(r[:, 4]):.0f}, "
              f"health {np.median(r[:, 5]):.0f}")
        print(f"placement loop parts (median sums): head {np.median(r[:, 6]):.0f} draw "
              f"{np.median(r[:, 7]):.0f} fixpoint {np.median(r[:, 8]):.0f} update {np.median(r[:, 9]):.0f}")
        print(f"jacobi (median sums): words {np.median(r[:, 10]):.0f} lens {np.median(r[:, 11]):.0f} "
              f"draws {np.median(r[:, 12]):.0f} cells {np.median(r[:, 13]):.0f} commit "
              f"{np.median(r[:, 14]):.0f}; sweeps median {np.median(r[:, 15]):.0f} max {r[:, 15].max()}")
        print(f"reset obs: tables+obs-par median {np.median(r[:, 16]):.0f}, crowded draws median "
              f"{np.median(r[:, 17]):.0f} mean {r[:, 17].mean():.0f}, store+tail median {np.median(r[:, 18]):.0f}")


if __name__ == '__main__':
    main()
