"""Fixtures for generate_maze (utils.py:120-212) and MazePlacementState
(state.py:385-619), produced by the REFERENCE itself (run in this container;
needs /root/reference): tests/golden/maze_gen.json.

  mazes:      generate_maze(rows, cols, start) after np.random.seed(seed):
              the maze and the legacy MT19937 state after it (position and
              a CRC-32 of the key).
  placements: MazePlacementState cases; per case, `resets` consecutive
              reset() calls after random.seed / np.random.seed: every agent's
              position, its rank inside its cell (Grid insertion order), the
              exception raised (if any) and the MT19937 state after.
  trajectories: the reference's MultiMazeNavigationSim example
              (examples/sim/multi_maze_navigation.py) under AllStepManager:
              scripted moves, per step obs / reward bits / dones / positions /
              MT19937 state, resets at __all__ or the horizon.
"""
import json
import os
import random
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'

MAZES = [
    # (rows, cols, start or None, seed)
    (5, 9, [1, 1], 0), (4, 4, None, 1), (16, 16, [0, 0], 2), (16, 16, None, 3),
    (7, 13, [3, 5], 4), (31, 31, [15, 15], 5), (64, 64, [10, 20], 6), (1, 1, [0, 0], 7),
    (2, 2, [0, 1], 8), (3, 3, None, 9), (9, 3, [4, 2], 10), (40, 25, None, 11),
    (12, 12, [5, 6], 24), (16, 16, [7, 8], 12345),
]

# agents: (id, encoding, initial_position or None)
def _tb(nb=5, nf=3, tgt_ip=None):
    return ([('target', 1, tgt_ip)] + [(f'barrier_agent{i}', 2, None) for i in range(nb)] +
            [(f'free_agent{i}', 3, None) for i in range(nf)])


PLACEMENTS = [
    dict(name='basic', rows=5, cols=8, agents=_tb(), overlapping={1: [3], 3: [3]},
         barrier=[2], free=[1, 3], seed=1, resets=8),
    dict(name='target_ip', rows=5, cols=8, agents=_tb(tgt_ip=[3, 2]), overlapping={1: [3], 3: [3]},
         barrier=[2], free=[1, 3], seed=2, resets=8),
    dict(name='cluster_scatter', rows=5, cols=8, agents=_tb(5, 5, [3, 2]), overlapping={1: [3], 3: [3]},
         barrier=[2], free=[1, 3], cluster=True, scatter=True, seed=24, resets=6),
    dict(name='cluster_scatter_no_overlap', rows=5, cols=8, agents=_tb(5, 5, [3, 2]),
         overlapping={1: [3], 3: [3]}, barrier=[2], free=[1, 3], cluster=True, scatter=True,
         no_overlap=True, seed=24, resets=6),
    dict(name='cluster_only', rows=7, cols=7, agents=_tb(8, 4), overlapping={1: [3], 3: [3]},
         barrier=[2], free=[1, 3], cluster=True, seed=5, resets=8),
    dict(name='scatter_only', rows=7, cols=9, agents=_tb(6, 6), overlapping={3: [3]},
         barrier=[2], free=[1, 3], scatter=True, seed=6, resets=8),
    dict(name='no_free', rows=5, cols=8, agents=[('target', 2, None)] + [(f'b{i}', 2, None) for i in range(5)],
         overlapping={}, barrier=[2], free=[], seed=7, resets=6),
    dict(name='ip_agents', rows=6, cols=6,
         agents=[('target', 1, None), ('ip0', 3, [0, 0]), ('b0', 2, None), ('ip1', 2, [5, 5]),
                 ('f0', 3, None), ('b1', 2, None)],
         overlapping={1: [3], 3: [3], 2: [2]}, barrier=[2], free=[1, 3], seed=8, resets=8),
    dict(name='ip_conflict', rows=5, cols=8,
         agents=[('target', 1, [3, 2]), ('ip_agent', 1, [3, 2])] + _tb()[1:],
         overlapping={1: [3], 3: [3]}, barrier=[2], free=[1, 3], seed=9, resets=2),
    dict(name='too_many', rows=4, cols=4,
         agents=[('target', 1, None)] + [(f'b{i}', 2, None) for i in range(10)] +
                [(f'f{i}', 3, None) for i in range(3)],
         overlapping={1: [3], 3: [3]}, barrier=[2], free=[1, 3], seed=10, resets=3),
    dict(name='both_sets', rows=6, cols=7,
         agents=[('target', 1, None), ('x0', 2, None), ('x1', 2, None), ('y0', 3, None)],
         overlapping={}, barrier=[2, 3], free=[1, 3], cluster=True, seed=11, resets=8),
    dict(name='shuffled', rows=6, cols=6, agents=_tb(6, 4), overlapping={1: [3], 3: [3]},
         barrier=[2], free=[1, 3], randomize=True, seed=12, resets=8),
    dict(name='multi_maze', rows=10, cols=10,
         agents=[('target', 1, None)] + [(f'navigator{i}', 2, None) for i in range(3)] +
                [(f'wall{i}', 3, None) for i in range(30)],
         overlapping={1: [2], 2: [2]}, barrier=[3], free=[1, 2], cluster=True, scatter=True,
         seed=13, resets=10),
    dict(name='multi_maze_plain', rows=8, cols=8,
         agents=[('target', 1, None)] + [(f'navigator{i}', 2, None) for i in range(4)] +
                [(f'wall{i}', 3, None) for i in range(20)],
         overlapping={1: [2], 2: [2]}, barrier=[3], free=[1, 2], seed=14, resets=10),
]


# TargetBarriersFreePlacementState (state.py:169-382): the same case shapes
TBF = [dict(c, name='tbf_' + c['name']) for c in PLACEMENTS
       if c['name'] in ('basic', 'target_ip', 'cluster_scatter', 'cluster_scatter_no_overlap',
                        'cluster_only', 'scatter_only', 'ip_agents', 'ip_conflict', 'both_sets',
                        'shuffled', 'multi_maze')]
TBF.append(dict(name='tbf_too_many', rows=3, cols=3,
                agents=[('target', 1, None)] + [(f'b{i}', 2, None) for i in range(10)],
                overlapping={}, barrier=[2], free=[1], cluster=True, seed=40, resets=2))


def mt_after():
    st = np.random.get_state()
    return int(st[2]), int(zlib.crc32(np.asarray(st[1], np.uint32).tobytes()))


def run_mazes(generate_maze):
    out = []
    for rows, cols, start, seed in MAZES:
        np.random.seed(seed)
        m = generate_maze(rows, cols, None if start is None else np.array(start))
        pos, crc = mt_after()
        out.append(dict(rows=rows, cols=cols, start=start, seed=seed,
                        maze=m.astype(int).reshape(-1).tolist(), mt_pos=pos, mt_crc=crc))
    return out


def run_placements(cases=None, cls_name='MazePlacementState'):
    from abmarl.sim.gridworld.grid import Grid
    from abmarl.sim.gridworld.agent import GridWorldAgent
    from abmarl.sim.gridworld import state as ref_state
    MazePlacementState = getattr(ref_state, cls_name)
    out = []
    for c in (PLACEMENTS if cases is None else cases):
        agents = {aid: GridWorldAgent(id=aid, encoding=enc,
                                      initial_position=None if ip is None else np.array(ip))
                  for aid, enc, ip in c['agents']}
        grid = Grid(c['rows'], c['cols'], overlapping={k: set(v) for k, v in c['overlapping'].items()})
        state = MazePlacementState(
            grid=grid, agents=agents, target_agent=agents['target'],
            barrier_encodings=set(c['barrier']), free_encodings=set(c['free']),
            cluster_barriers=c.get('cluster', False), scatter_free_agents=c.get('scatter', False),
            no_overlap_at_reset=c.get('no_overlap', False),
            randomize_placement_order=c.get('randomize', False))
        random.seed(c['seed'])
        np.random.seed(c['seed'])
        ids = [a[0] for a in c['agents']]
        resets = []
        for _ in range(c['resets']):
            rec = {}
            try:
                state.reset()
                rec['raised'] = None
            except AssertionError:
                rec['raised'] = 'AssertionError'
            except RuntimeError:
                rec['raised'] = 'RuntimeError'
            rank = {}
            for r in range(c['rows']):
                for cc in range(c['cols']):
                    for k, aid in enumerate(grid[r, cc]):
                        rank[aid] = (r, cc, k)
            rec['cells'] = [list(rank[aid]) if aid in rank else None for aid in ids]
            rec['order'] = list(state.agents) if c.get('randomize', False) else None
            rec['mt_pos'], rec['mt_crc'] = mt_after()
            resets.append(rec)
            if rec['raised']:
                break
        out.append(dict(c, resets_out=resets))
    return out


TRAJ = [
    dict(name='mm_10', rows=10, cols=10, navigators=3, walls=30, view=2, cluster=True, scatter=True,
         seed=31, steps=40, horizon=20),
    dict(name='mm_8', rows=8, cols=8, navigators=2, walls=15, view=3, cluster=False, scatter=False,
         seed=32, steps=40, horizon=15),
]


def build_multi_maze(t, sim_cls, nav_cls, gw_agent_cls):
    """The MultiMazeNavigation layout of TRAJ entry t (reference example
    classes or this repository's)."""
    agents = {'target': gw_agent_cls(id='target', encoding=1)}
    for i in range(t['navigators']):
        agents[f'navigator{i}'] = nav_cls(id=f'navigator{i}', encoding=2, view_range=t['view'])
    for i in range(t['walls']):
        agents[f'wall{i}'] = gw_agent_cls(id=f'wall{i}', encoding=3, blocking=True)
    return sim_cls.build_sim(t['rows'], t['cols'], agents=agents, overlapping={1: {2}, 2: {2}},
                             target_agent=agents['target'], barrier_encodings={3},
                             free_encodings={1, 2}, cluster_barriers=t['cluster'],
                             scatter_free_agents=t['scatter'])


def multi_maze_actions(t):
    rng = np.random.default_rng(t['seed'])
    return rng.integers(-1, 2, size=(t['steps'], t['navigators'], 2)).tolist()


def run_multi_maze(t, sim, manager_cls):
    """AllStepManager episodes of sim: per step the navigators' obs, reward
    bits, dones, every agent's position and the MT19937 state."""
    key = 'position_centered_encoding'
    man = manager_cls(sim)
    np.random.seed(t['seed'])
    navs = [f'navigator{i}' for i in range(t['navigators'])]
    acts = multi_maze_actions(t)
    rec = []
    obs = man.reset()
    ep_t = 0
    for step in range(t['steps']):
        entry = dict(obs={k: np.asarray(v[key]).astype(int).tolist() for k, v in obs.items()})
        ad = {n: {'move': np.array(acts[step][i])} for i, n in enumerate(navs) if n not in man.done_agents}
        obs, rew, done, _ = man.step(ad)
        ep_t += 1
        entry['reward'] = {k: np.float64(v).view(np.uint64).item() for k, v in rew.items()}
        entry['done'] = {k: bool(v) for k, v in done.items()}
        entry['pos'] = {k: np.asarray(a.position).astype(int).tolist() for k, a in sim.agents.items()}
        entry['mt_pos'], entry['mt_crc'] = mt_after()
        entry['reset'] = bool(done['__all__'] or ep_t >= t['horizon'])
        rec.append(entry)
        if entry['reset']:
            obs = man.reset()
            ep_t = 0
    return rec


def main():
    sys.path.insert(0, HERE)
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    from abmarl.sim.gridworld.utils import generate_maze
    from abmarl.examples.sim.multi_maze_navigation import MultiMazeNavigationSim, MultiMazeNavigationAgent
    from abmarl.sim.gridworld.agent import GridWorldAgent
    from abmarl.managers import AllStepManager
    traj = []
    for t in TRAJ:
        sim = build_multi_maze(t, MultiMazeNavigationSim, MultiMazeNavigationAgent, GridWorldAgent)
        traj.append(dict(t, steps_out=run_multi_maze(t, sim, AllStepManager)))
    data = dict(python=sys.version.split()[0], numpy=np.__version__,
                mazes=run_mazes(generate_maze), placements=run_placements(), trajectories=traj,
                tbf=run_placements(TBF, 'TargetBarriersFreePlacementState'))
    path = os.path.join(HERE, 'maze_gen.json')
    with open(path, 'w') as f:
        json.dump(data, f, separators=(',', ':'))
    print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
