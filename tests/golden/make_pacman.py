"""Generate Pacman golden trajectories by running the REFERENCE PacmanSim
(examples/sim/pacman.py) under its AllStepManager in this container.

Output: tests/golden/pacman_<case>.npz — inputs (seeds, actions) and the
reference's outputs per step for the Agents (pacman and the baddies, dict
order): absolute-encoding observations, rewards, dones, __all__, positions,
orientations, pacman's health, which food is left, and the RNG position +
key digest.  These are data fixtures; no reference source leaves
/root/reference.

Harness contract (as tests/golden/make_golden.py): one sim + manager per env
with its own np.random stream (seed, get/set_state); the state components
(a set in smart.py:37) pinned to Position, Orientation, Health; identical
int actions from an independent RandomState; reset after '__all__' or at the
horizon without reseeding.  The reference cannot run turn-based (pacman.py:82
indexes action_dict['pacman']), so these fixtures are AllStepManager only.

Run:  python tests/golden/make_pacman.py      (needs /root/reference)
"""
import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('ABMARL_REFERENCE', '/root/reference')
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

CASES = [
    # BASELINE config 5's map (four baddies), default reward scheme
    dict(name='pacman_4', baddies=[[9, 5], [9, 8], [9, 10], [9, 12]], n_envs=6, n_steps=150,
         horizon=60, seed_base=501, reward_scheme=None),
    # the full pacman.txt (ten baddies), examples/rllib_pacman.py's scheme + kill
    dict(name='pacman_10', baddies=None, n_envs=4, n_steps=120, horizon=80, seed_base=777,
         reward_scheme={'bad_move': 0, 'entropy': -0.01, 'eat_food': 0.05, 'kill': 1, 'die': -1}),
    # AllStepManager(randomize_action_input=True): the baddies move in the
    # shuffled action dict's order (Python's random, per env)
    dict(name='pacman_shuffle_act', baddies=None, n_envs=4, n_steps=120, horizon=80, seed_base=881,
         reward_scheme={'bad_move': -0.1, 'entropy': -0.01, 'eat_food': 0.05, 'kill': 1, 'die': -1},
         randomize_action_input=True),
]


def build_reference(c):
    from abmarl.examples.sim.pacman import (PacmanSim, PacmanAgent, WallAgent, FoodAgent,
                                            BaddieAgent)
    from abmarl.sim.gridworld.state import PositionState, OrientationState, HealthState
    from abmarl.managers import AllStepManager
    from abmarl_amd.examples.pacman import pacman_grid
    registry = {
        'P': lambda n: PacmanAgent(id='pacman', encoding=1),
        'W': lambda n: WallAgent(id=f'wall_{n}', encoding=2),
        'F': lambda n: FoodAgent(id=f'food_{n}', encoding=3),
        'B': lambda n: BaddieAgent(id=f'baddie_{n}', encoding=4),
    }
    kw = {}
    if c['reward_scheme'] is not None:
        kw['reward_scheme'] = c['reward_scheme']
    sim = PacmanSim.build_sim_from_array(
        pacman_grid(c['baddies']), registry,
        states={'PositionState', 'OrientationState', 'HealthState'},
        observers={'AbsoluteEncodingObserver'}, overlapping={1: {3, 4}, 4: {3, 4}}, **kw)
    pos = [s for s in sim._states if isinstance(s, PositionState)][0]
    ori = [s for s in sim._states if isinstance(s, OrientationState)][0]
    hea = [s for s in sim._states if isinstance(s, HealthState)][0]
    sim._states = [pos, ori, hea]
    return AllStepManager(sim, randomize_action_input=c.get('randomize_action_input', False)), FoodAgent


def run_case(c):
    from abmarl.sim import Agent
    T, E = c['n_steps'], c['n_envs']
    managers, food_cls = zip(*[build_reference(c) for _ in range(E)])
    food_cls = food_cls[0]
    ids = list(managers[0].agents.keys())
    agents_ix = [i for i, a in enumerate(managers[0].agents.values()) if isinstance(a, Agent)]
    food_ix = [i for i, a in enumerate(managers[0].agents.values()) if isinstance(a, food_cls)]
    NA = len(agents_ix)
    H, W = managers[0].sim.grid.rows, managers[0].sim.grid.cols
    c = dict(c, seeds=[c['seed_base'] + e for e in range(E)], agent_index=agents_ix,
             food_index=food_ix, n_entities=len(ids))
    act = np.random.RandomState(c['seed_base'] + 1).randint(0, 5, size=(T, E, NA)).astype(np.int8)

    def obs_array(d):
        out = np.full((NA, H, W), -2, dtype=np.int8)
        ret = np.zeros(NA, dtype=np.uint8)
        for j, i in enumerate(agents_ix):
            if ids[i] in d:
                out[j] = d[ids[i]]['absolute_encoding']
                ret[j] = 1
        return out, ret

    def snapshot(m):
        ag = list(m.agents.values())
        pos = np.array([ag[i].position for i in agents_ix], dtype=np.int8)
        ori = np.array([ag[i].orientation for i in agents_ix], dtype=np.int8)
        food = np.array([ag[i].active for i in food_ix], dtype=np.uint8)
        return pos, ori, food, float(m.sim.pacman.health)

    import random
    if c.get('randomize_action_input'):
        c['py_seeds'] = [(c['seed_base'] * 7919 + e) & 0xFFFFFFFF for e in range(E)]
    rng_states, py_states, obs0 = [], [], np.zeros((E, NA, H, W), np.int8)
    for e in range(E):
        np.random.seed(c['seeds'][e])
        if 'py_seeds' in c:
            random.seed(c['py_seeds'][e])
        obs0[e], _ = obs_array(managers[e].reset())
        rng_states.append(np.random.get_state())
        py_states.append(random.getstate())
    out = dict(
        obs=np.full((T, E, NA, H, W), -2, dtype=np.int8),
        returned=np.zeros((T, E, NA), np.uint8),
        reward=np.zeros((T, E, NA), np.float64),
        done=np.ones((T, E, NA), np.uint8),
        all_done=np.zeros((T, E), np.uint8),
        pos=np.zeros((T, E, NA, 2), np.int8),
        orient=np.zeros((T, E, NA), np.int8),
        food=np.zeros((T, E, len(food_ix)), np.uint8),
        pac_health=np.zeros((T, E), np.float64),
        mt_pos=np.zeros((T, E), np.int16),
        mt_crc=np.zeros((T, E), np.uint32),
        reset_mask=np.zeros((T, E), np.uint8),
        reset_obs=np.full((T, E, NA, H, W), -2, dtype=np.int8),
    )
    steps = [0] * E
    for t in range(T):
        for e in range(E):
            m = managers[e]
            np.random.set_state(rng_states[e])
            random.setstate(py_states[e])
            adict = {ids[i]: {'move': int(act[t, e, j])} for j, i in enumerate(agents_ix)
                     if ids[i] not in m.done_agents}
            o, r, d, _ = m.step(adict)
            steps[e] += 1
            out['obs'][t, e], out['returned'][t, e] = obs_array(o)
            for j, i in enumerate(agents_ix):
                if ids[i] in r:
                    out['reward'][t, e, j] = r[ids[i]]
                    out['done'][t, e, j] = int(bool(d[ids[i]]))
            out['all_done'][t, e] = int(bool(d['__all__']))
            (out['pos'][t, e], out['orient'][t, e], out['food'][t, e],
             out['pac_health'][t, e]) = snapshot(m)
            st = np.random.get_state()
            out['mt_pos'][t, e] = st[2]
            out['mt_crc'][t, e] = zlib.crc32(np.ascontiguousarray(st[1], dtype=np.uint32).tobytes())
            if d['__all__'] or steps[e] >= c['horizon']:
                ro = m.reset()
                steps[e] = 0
                out['reset_mask'][t, e] = 1
                out['reset_obs'][t, e], _ = obs_array(ro)
            rng_states[e] = np.random.get_state()
            py_states[e] = random.getstate()
    path = os.path.join(HERE, c['name'] + '.npz')
    np.savez_compressed(path, case=json.dumps(c), actions=act, obs0=obs0, **out)
    deaths = int(((out['pac_health'] == 0) & (out['all_done'] == 1)).sum())
    eaten = int(len(food_ix) * E * T - out['food'].sum())
    print(f"{c['name']}: {T} steps x {E} envs, {NA} agents, resets={int(out['reset_mask'].sum())}, "
          f"deaths={deaths}, food-steps eaten={eaten} -> {os.path.getsize(path)} B")


def main():
    sys.path.insert(0, HERE)
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    only = sys.argv[1:]
    for c in CASES:
        if not only or c['name'] in only:
            run_case(c)


if __name__ == '__main__':
    main()
