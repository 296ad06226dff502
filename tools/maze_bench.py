"""Time generate_maze and MazePlacementState.reset on the device (one wave
per env, gw_maze.inc) against the C oracle on one host core.

    python tools/maze_bench.py [--envs 4096] [--rows 16] [--cols 16] [--iters 5]

Prints one JSON line: device ms per call, mazes (or resets) per second, and
the oracle's per-env time.  The MultiMazeNavigation layout: target + 3
navigators (free) + 30 walls (barrier), cluster + scatter.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abmarl_amd import _abi  # noqa: E402
from abmarl_amd.engine import GridWorldEngine  # noqa: E402
from abmarl_amd.sim.gridworld.agent import GridWorldAgent  # noqa: E402
from abmarl_amd.sim.gridworld.compile import agent_spec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--envs', type=int, default=4096)
    ap.add_argument('--rows', type=int, default=16)
    ap.add_argument('--cols', type=int, default=16)
    ap.add_argument('--iters', type=int, default=5)
    a = ap.parse_args()
    agents = [GridWorldAgent(id='target', encoding=1)] + \
        [GridWorldAgent(id=f'n{i}', encoding=2) for i in range(3)] + \
        [GridWorldAgent(id=f'w{i}', encoding=3, blocking=True) for i in range(30)]
    cc = _abi.CompiledConfig(a.rows, a.cols, [agent_spec(x) for x in agents], _abi.GW_SIM_TEAM_BATTLE,
                             {1: 1 << 2, 2: (1 << 1) | (1 << 2)}, {})
    cc.cfg.all_lanes = 1
    eng = GridWorldEngine(cc, a.envs, seeds=list(range(a.envs)))
    start = torch.full((a.envs, 2), -1, dtype=torch.int32, device=eng.device)
    out = torch.empty((a.envs, a.rows, a.cols), dtype=torch.int8, device=eng.device)
    res = {}
    for what in ('generate_maze', 'maze_reset'):
        def call():
            if what == 'generate_maze':
                eng.generate_maze(start, out)
            else:
                eng.maze_reset(0, {3}, {1, 2}, cluster_barriers=True, scatter_free_agents=True)
        call()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.iters):
            call()
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.iters
        res[what] = dict(ms_per_call=round(ms, 4), per_s=round(a.envs / ms * 1e3, 1))
    # oracle: one host core, a bounded sample of envs
    from oracle import oracle
    n = min(64, a.envs)
    t = time.perf_counter()
    for e in range(n):
        mt = oracle.mt_state(e)
        oracle.maze_place(cc, 0, [3], [1, 2], mt, cluster=True, scatter=True)
    cpu = (time.perf_counter() - t) / n
    res['oracle_maze_reset_ms_per_env'] = round(cpu * 1e3, 4)
    res['config'] = dict(envs=a.envs, rows=a.rows, cols=a.cols, entities=len(agents))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
