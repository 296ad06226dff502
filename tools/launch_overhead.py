"""Where the wall time of the headline's one timed 20-step launch goes
(bench.py run_rollout's timed region), measured piece by piece after the
same pre-roll: host time of each event record and of the gw_rollout call,
the kernel's event time, and the wall from the synchronize before to the
synchronize after.  Each trial starts from an idle, synchronized GPU, as
the timed region does.

    python tools/launch_overhead.py [--trials 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402
from abmarl_amd.examples.workloads import team_battle_sim  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trials', type=int, default=8)
    ap.add_argument('--envs', type=int, default=4096)
    a = ap.parse_args()
    cc = team_battle_sim().compiled()
    E, H, F = a.envs, 200, 20
    eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
    eng.reset()
    eng.all_done.zero_()
    eng.set_state(steps=torch.as_tensor((np.arange(E) * H // E).astype(np.int32), device=eng.device))
    acts = torch.empty((100,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
    out = eng.rollout_buffers(100)
    t = 0
    for _ in range(10):
        for s in range(100):
            eng.random_actions(5, t + s, out=acts[s])
        eng.rollout(acts, horizon=H, skip_done_obs=True, out=out)
        t += 100
    torch.cuda.synchronize()
    rows = []
    for k in range(a.trials):
        for s in range(F):
            eng.random_actions(5, t + s, out=acts[s])
        t += F
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        ev1.record()                             # created outside the timed region (bench.py)
        launch = eng.rollout_launcher(acts[:F], horizon=H, skip_done_obs=True, out=out)
        torch.cuda.synchronize()
        time.sleep(0.002)
        w0 = time.perf_counter()
        ev0.record()
        w1 = time.perf_counter()
        launch()
        w2 = time.perf_counter()
        ev1.record()
        w3 = time.perf_counter()
        torch.cuda.synchronize()
        w4 = time.perf_counter()
        rows.append(dict(record0_us=(w1 - w0) * 1e6, rollout_call_us=(w2 - w1) * 1e6,
                         record1_us=(w3 - w2) * 1e6, sync_wait_us=(w4 - w3) * 1e6,
                         wall_us=(w4 - w0) * 1e6, event_us=ev0.elapsed_time(ev1) * 1e3))
    med = {k: round(float(np.median([r[k] for r in rows])), 1) for k in rows[0]}
    print(json.dumps({'envs': E, 'steps_per_launch': F, 'trials': a.trials, 'median': med,
                      'all': [{k: round(v, 1) for k, v in r.items()} for r in rows]}))


if __name__ == '__main__':
    main()
