"""Generate golden trajectories by running the REFERENCE (gillette7/Abmarl at
/root/reference) in this container.

Output: tests/golden/<case>.npz — inputs (config, seeds, actions) and the
reference's outputs (obs, rewards, dones, __all__, positions, health, RNG
position + key digest) per step.  These are data fixtures; the reference
source never leaves /root/reference.

Harness contract:
  * one reference sim + AllStepManager per env, each with its own numpy
    legacy RNG stream: np.random.seed(seed_e), isolated with get/set_state;
  * the SmartGridWorldSimulation state components, stored by the reference
    in a Python set (smart.py:37), are pinned to an explicit order;
  * identical int actions are fed to every env (generated here with an
    independent RandomState, stored in the fixture);
  * auto-reset after a step whose '__all__' is True or when the env reached
    the horizon, without reseeding (the RNG stream continues).

Run:  python tests/golden/make_golden.py      (needs /root/reference)
"""
import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('ABMARL_REFERENCE', '/root/reference')

# static walls for tb_walls: two bars and a few pillars
WALLS_12 = [[2, c] for c in range(2, 6)] + [[r, 8] for r in range(5, 10)] + \
    [[6, 3], [9, 5], [4, 10], [10, 1]]

CASES = [
    # tiny grid that forces stacks, kills and episode ends
    dict(name='tb_small', rows=8, cols=8, n_agents=8, n_teams=2, n_envs=6, n_steps=120,
         horizon=50, seed_base=11),
    # three teams, cross-team overlap (mixed-encoding cells => the observer's
    # choice value matters), observe_self=False, partial accuracy, wider ranges
    dict(name='tb_mixed', rows=7, cols=9, n_agents=12, n_teams=3, n_envs=6, n_steps=120,
         horizon=40, seed_base=101, overlap={1: [1, 2], 2: [2], 3: [3, 1]},
         attack_mapping={1: [2, 3], 2: [1, 3], 3: [1, 2]}, observe_self=False,
         agent=dict(move_range=1, attack_range=2, attack_strength=0.6, attack_accuracy=0.7,
                    view_range=2)),
    # health first at reset, no_overlap_at_reset, some initial positions/health
    dict(name='tb_order', rows=6, cols=6, n_agents=10, n_teams=2, n_envs=5, n_steps=100,
         horizon=30, seed_base=7, state_order='health_position', no_overlap_at_reset=True,
         initial_positions={0: [0, 0], 3: [5, 5], 4: [0, 0]}, initial_health={1: 1.0, 2: 0.25}),
    # the headline configuration (32x32, 64 agents, 2 teams), past one horizon
    dict(name='tb_32', rows=32, cols=32, n_agents=64, n_teams=2, n_envs=2, n_steps=230,
         horizon=200, seed_base=1000003),
    # the reference example's layout: 24 agents, 4 teams on 4 corner cells
    dict(name='tb_corners', rows=8, cols=8, n_agents=24, n_teams=4, n_envs=3, n_steps=80,
         horizon=60, seed_base=5, corners=True),
    # blocking: static walls (encoding 3, blocking, overlap nothing) from an
    # array plus blocking fighters; attack range 2 so the attack mask matters
    dict(name='tb_walls', rows=12, cols=12, n_agents=16, n_teams=2, n_envs=4, n_steps=120,
         horizon=60, seed_base=77, walls=WALLS_12, wall_encoding=3, blocking=[0, 3, 5, 10],
         agent=dict(move_range=1, attack_range=2, attack_strength=0.5, attack_accuracy=0.9,
                    view_range=3)),
    # MazeNavigation on the reference's own examples/maze.txt
    # (examples/rllib_maze_navigation.py: view 2, walls blocking)
    dict(name='maze_file', kind='maze', maze='maze.txt', n_envs=4, n_steps=150, horizon=100,
         seed_base=3, agent=dict(move_range=1, view_range=2)),
    # ReachTheTarget (examples/rllib_reach_the_target.py layout: 10 barriers,
    # runners in the corners, the target in the center; view ranges equal)
    dict(name='rtt_7', kind='rtt', rows=7, cols=7, n_barriers=10, n_runners=4, n_envs=4,
         n_steps=120, horizon=40, seed_base=21, corners=True,
         runner=dict(move_range=2, view_range=3, initial_health=1),
         target=dict(view_range=3, attack_range=1, attack_strength=1, attack_accuracy=1)),
    # larger, random placement and health, partial accuracy, 2 attacks per cell
    dict(name='rtt_16', kind='rtt', rows=16, cols=16, n_barriers=30, n_runners=20, n_envs=3,
         n_steps=100, horizon=60, seed_base=33,
         runner=dict(move_range=2, view_range=3),
         target=dict(view_range=3, attack_range=2, attack_strength=0.6, attack_accuracy=0.8,
                     simultaneous_attacks=2)),
    # crowded: runners placed on the target's cell get killed there by its
    # center attack, then removed again in the move pass -> KeyError (recorded)
    dict(name='rtt_double', kind='rtt', rows=5, cols=5, n_barriers=3, n_runners=14, n_envs=6,
         n_steps=80, horizon=25, seed_base=44,
         runner=dict(move_range=1, view_range=2, initial_health=1),
         target=dict(view_range=2, attack_range=1, attack_strength=1, attack_accuracy=1)),
    # BASELINE config 4's size: 64x64, 128 barriers, 127 runners, the target
    # in the center (as in the reference example); 256 entities, so the
    # engine runs it on its workgroup-per-env kernel
    dict(name='rtt_64', kind='rtt', rows=64, cols=64, n_barriers=128, n_runners=127, n_envs=2,
         n_steps=60, horizon=40, seed_base=64, target_center=True,
         runner=dict(move_range=2, view_range=3, initial_health=1),
         target=dict(view_range=3, attack_range=1, attack_strength=1, attack_accuracy=1)),
    # MazeNavigation 16x16 from generate_maze (utils.py:120-212), N and T on passages
    # TeamBattle with the target done components (done.py:59-137): each
    # fighter hunts the next one of the other team (TargetDestroyedDone) or
    # chases it (TargetAgentDone)
    dict(name='tb_destroy', rows=7, cols=7, n_agents=10, n_teams=2, n_envs=5, n_steps=120,
         horizon=60, seed_base=61, dones=['ActiveDone', 'TargetDestroyedDone'],
         target_mapping={i: (i + 1) % 10 for i in range(10)},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.8,
                    view_range=2)),
    dict(name='tb_chase', rows=6, cols=6, n_agents=8, n_teams=2, n_envs=5, n_steps=120,
         horizon=50, seed_base=71, dones=['TargetAgentDone'],
         target_mapping={i: (i + 3) % 8 for i in range(8)}, overlap={1: [1, 2], 2: [2]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.3, attack_accuracy=1,
                    view_range=2)),
    # TrafficCorridor: the reference example itself (examples/rllib_traffic_corridor_2_teams.py)
    dict(name='traffic_ex', kind='traffic', n_envs=6, n_steps=150, horizon=40, seed_base=91,
         grid=['GWWWR', 'r___g', 'GWWWR'],
         target_mapping={'red4': 'red_target', 'red11': 'red_target', 'green0': 'green_target',
                         'green7': 'green_target'}),
    # a longer two-lane corridor with more traffic
    dict(name='traffic_9', kind='traffic', n_envs=4, n_steps=150, horizon=60, seed_base=93,
         grid=['G_WWWWW_R', 'G_______R', 'r___W___g', 'G_______R', 'G_WWWWW_R'], targets='team'),
    # the reference's own ReachTheTarget example (examples/rllib_reach_the_target.py):
    # runners see 3 cells, the target 7 (different view ranges)
    dict(name='rtt_7_views', kind='rtt', rows=7, cols=7, n_barriers=10, n_runners=4, n_envs=4,
         n_steps=120, horizon=40, seed_base=27, corners=True,
         runner=dict(move_range=2, view_range=3, initial_health=1),
         target=dict(view_range=7, attack_range=1, attack_strength=1, attack_accuracy=1)),
    # the same example's layout at 16x16 with its own view-range rule
    # (rllib_reach_the_target.py:22-31: runners grid_size / 2, the target
    # grid_size): windows of 17x17 and 33x33 cells
    dict(name='rtt_16_example', kind='rtt', rows=16, cols=16, n_barriers=10, n_runners=4, n_envs=3,
         n_steps=100, horizon=40, seed_base=29, corners=True,
         runner=dict(move_range=2, view_range=8, initial_health=1),
         target=dict(view_range=16, attack_range=1, attack_strength=1, attack_accuracy=1)),
    # TeamBattle with view ranges 1, 2 and 3 mixed, blocking walls and fighters
    dict(name='tb_views', rows=10, cols=10, n_agents=18, n_teams=2, n_envs=4, n_steps=120,
         horizon=60, seed_base=81, views=[1, 3, 2], walls=[[2, c] for c in range(2, 7)] +
         [[r, 7] for r in range(4, 9)], wall_encoding=3, blocking=[0, 4, 9, 13],
         agent=dict(move_range=1, attack_range=2, attack_strength=0.5, attack_accuracy=0.9,
                    view_range=3)),
    dict(name='maze_16', kind='maze', maze='generate:16:16:2024', n_envs=4, n_steps=200,
         horizon=150, seed_base=9, agent=dict(move_range=1, view_range=2)),
    # TeamBattle beyond one wavefront: 128 fighters (the engine's workgroup-
    # per-env kernel), the example's BattleAgent, 2 teams on 24x24
    dict(name='tb_128', rows=24, cols=24, n_agents=128, n_teams=2, n_envs=2, n_steps=140,
         horizon=100, seed_base=128),
    # 100 fighters in 4 teams on 16x16: accuracy < 1, attack range 2, two
    # stacked attacks, cross-team overlap, observe_self=False
    dict(name='tb_100', rows=16, cols=16, n_agents=100, n_teams=4, n_envs=2, n_steps=120,
         horizon=70, seed_base=100, overlap={1: [1, 3], 2: [2], 3: [3], 4: [4, 2]},
         stacked_attacks=True, observe_self=False,
         agent=dict(move_range=1, attack_range=2, attack_strength=0.4, attack_accuracy=0.8,
                    view_range=2, simultaneous_attacks=2)),
    # PositionState(randomize_placement_order=True): Python's random.shuffle of
    # the agents dict before every placement (state.py:97-101), shared initial
    # cells within a team so the shuffled insertion order shows in the
    # crowded-cell draws; per-env Python random streams (py_seeds)
    dict(name='tb_shuffle', rows=8, cols=8, n_agents=12, n_teams=2, n_envs=4, n_steps=150,
         horizon=30, seed_base=55, randomize_placement_order=True,
         initial_positions={0: [0, 0], 2: [0, 0], 5: [3, 3], 7: [3, 3]}),
    # AllStepManager(randomize_action_input=True): the action dict shuffled
    # with Python's random every step (all_step_manager.py:62-65), so the
    # attack and move passes run in that order; dense, accuracy < 1
    dict(name='tb_shuffle_act', rows=7, cols=7, n_agents=16, n_teams=2, n_envs=4, n_steps=150,
         horizon=40, seed_base=57, randomize_action_input=True,
         overlap={1: [1, 2], 2: [2, 1]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.6, attack_accuracy=0.7,
                    view_range=2)),
    # the same for the ReachTheTarget and TrafficCorridor programs: runners move
    # (and enter cells) in the shuffled dict's order
    dict(name='rtt_shuffle_act', kind='rtt', rows=9, cols=9, n_barriers=12, n_runners=24, n_envs=4,
         n_steps=120, horizon=40, seed_base=61, randomize_action_input=True,
         runner=dict(move_range=1, view_range=2),
         target=dict(view_range=2, attack_range=1, attack_strength=0.6, attack_accuracy=0.8,
                     simultaneous_attacks=2)),
    dict(name='traffic_shuffle_act', kind='traffic', n_envs=4, n_steps=150, horizon=60, seed_base=63,
         randomize_action_input=True,
         grid=['G_WWWWW_R', 'G_______R', 'r___W___g', 'G_______R', 'G_WWWWW_R'], targets='team'),
    # AmmoAgent fighters (agent.py:291-322) + AmmoState (state.py:644-656):
    # up to 3 attacks a step against 1..5 rounds of ammo, so the ammo filter
    # (actor.py:343-351) keeps choice(attacked, ammo, replace=False) of the
    # attacked list, and attacks at 0 ammo still draw the permutation
    dict(name='tb_ammo', rows=7, cols=7, n_agents=14, n_teams=2, n_envs=4, n_steps=140, horizon=45,
         seed_base=201, ammo=[1, 3, 2], overlap={1: [1, 2], 2: [2, 1]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.9,
                    view_range=2)),
    # a negative initial_ammo: AmmoState.reset assigns it through the ammo
    # setter, which clamps to 0 (agent.py:308-311), so those fighters' attacks
    # keep choice(attacked, 0) = nothing and cost -0.1
    dict(name='tb_ammo_negative', rows=7, cols=7, n_agents=14, n_teams=2, n_envs=4, n_steps=120,
         horizon=40, seed_base=217, ammo=[-2, 1, 0, 3], overlap={1: [1, 2], 2: [2, 1]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.9,
                    view_range=2)),
    # several attacks a step (simultaneous_attacks 3, stacked or not), so the
    # ammo filter draws its permutation over longer attacked lists.  The
    # reference's TeamBattleSim.step tests `not attacked_agents`
    # (team_battle_example.py:41), which raises ValueError on the numpy array
    # _subset_attackables returns for two or more picks; these fixtures run
    # the example with that test as `len(attacked_agents) == 0` (len_fix),
    # the program's meaning, everything else the reference's own code
    dict(name='tb_ammo_multi', rows=7, cols=7, n_agents=14, n_teams=2, n_envs=4, n_steps=140,
         horizon=45, seed_base=207, ammo=[1, 3, 5, 2], attack_max=3, len_fix=True,
         overlap={1: [1, 2], 2: [2, 1]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.9,
                    view_range=2, simultaneous_attacks=3)),
    dict(name='tb_ammo_stacked', rows=6, cols=6, n_agents=10, n_teams=2, n_envs=4, n_steps=120,
         horizon=40, seed_base=203, ammo=[2, 4], attack_max=2, stacked_attacks=True, len_fix=True,
         agent=dict(move_range=1, attack_range=2, attack_strength=0.4, attack_accuracy=1,
                    view_range=2, simultaneous_attacks=2)),
    # the reference's own TeamBattleSim with simultaneous_attacks 3: whenever
    # _subset_attackables returns np.random.choice's array of two or more
    # agents (actor.py:412-414), `not attacked_agents` (team_battle_example.py:41)
    # raises ValueError -- recorded per env-step like the KeyError (err = 2),
    # after the attack's damage and draws; the env is then reset
    dict(name='tb_value_error', rows=7, cols=7, n_agents=14, n_teams=2, n_envs=6, n_steps=140,
         horizon=45, seed_base=211, attack_max=3, overlap={1: [1, 2], 2: [2, 1]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.9,
                    view_range=2, simultaneous_attacks=3)),
    # stacked attacks (choice with replacement: an array for any candidate
    # count) and AmmoAgents, whose filter turns a longer list into a list
    dict(name='tb_value_error_ammo', rows=6, cols=6, n_agents=10, n_teams=2, n_envs=6, n_steps=120,
         horizon=40, seed_base=213, ammo=[1, 3], attack_max=2, stacked_attacks=True,
         agent=dict(move_range=1, attack_range=2, attack_strength=0.4, attack_accuracy=1,
                    view_range=2, simultaneous_attacks=2)),
    # ReachTheTarget whose target is an AmmoAgent (SelectiveAttackActor: two
    # attacks per cell of its window) and an AmmoState beside the example's states
    dict(name='rtt_ammo', kind='rtt', rows=9, cols=9, n_barriers=8, n_runners=20, n_envs=4,
         n_steps=120, horizon=40, seed_base=205, target_ammo=6,
         runner=dict(move_range=1, view_range=2, initial_health=1),
         target=dict(view_range=2, attack_range=1, attack_strength=1, attack_accuracy=0.9,
                     simultaneous_attacks=2)),
]

DEFAULT_AGENT = dict(move_range=1, attack_range=1, attack_strength=1, attack_accuracy=1,
                     view_range=3)


def maze_array(spec):
    """The maze as a list of rows of characters ('W', 'N', 'T', '_')."""
    if spec.startswith('generate:'):
        from abmarl.sim.gridworld.utils import generate_maze
        _, rows, cols, seed = spec.split(':')
        np.random.seed(int(seed))
        m = generate_maze(int(rows), int(cols))
        free = [(r, c) for r in range(m.shape[0]) for c in range(m.shape[1]) if m[r, c] == 0]
        out = [['W' if v else '_' for v in row] for row in m]
        # target: the nearest passage at Chebyshev distance >= 3 from the
        # navigator, so random walks reach it within an episode
        nr, nc = free[0]
        tr, tc = min((p for p in free if max(abs(p[0] - nr), abs(p[1] - nc)) >= 3),
                     key=lambda p: (abs(p[0] - nr) + abs(p[1] - nc), p))
        out[nr][nc], out[tr][tc] = 'N', 'T'
        return out
    path = os.path.join(REF, 'examples', spec)
    return [line.split(' ') for line in open(path).read().splitlines()]


def full_case(case):
    c = dict(case)
    if c.get('kind') in ('traffic', 'rtt') and c.get('randomize_action_input', False):
        c['py_seeds'] = [(c['seed_base'] * 7919 + e) & 0xFFFFFFFF for e in range(c['n_envs'])]
    if c.get('kind') == 'traffic':
        c['seeds'] = [(c['seed_base'] + e) & 0xFFFFFFFF for e in range(c['n_envs'])]
        c['action_seed'] = 1234 + c['seed_base']
        c['agent'] = dict(move_range=1, view_range=3)
        return c
    if c.get('kind') == 'rtt':
        c['seeds'] = [(c['seed_base'] + e) & 0xFFFFFFFF for e in range(c['n_envs'])]
        c['action_seed'] = 1234 + c['seed_base']
        c['agent'] = dict(view_range=max(c['runner']['view_range'], c['target']['view_range']))
        return c
    if c.get('kind') == 'maze':
        c['maze'] = maze_array(c['maze'])
        c.setdefault('state_order', 'position_health')
        c['seeds'] = [(c['seed_base'] + e) & 0xFFFFFFFF for e in range(c['n_envs'])]
        c['action_seed'] = 1234 + c['seed_base']
        return c
    c.setdefault('kind', 'tb')
    c.setdefault('walls', [])
    c.setdefault('blocking', [])
    nt = c['n_teams']
    c.setdefault('overlap', {t: [t] for t in range(1, nt + 1)})
    c.setdefault('attack_mapping', {t: [u for u in range(1, nt + 1) if u != t]
                                    for t in range(1, nt + 1)})
    c.setdefault('observe_self', True)
    c.setdefault('no_overlap_at_reset', False)
    c.setdefault('stacked_attacks', False)
    c.setdefault('state_order', 'position_health')
    c.setdefault('initial_positions', {})
    c.setdefault('initial_health', {})
    c.setdefault('agent', DEFAULT_AGENT)
    c.setdefault('dones', ['OneTeamRemainingDone'])
    c.setdefault('randomize_placement_order', False)
    c.setdefault('randomize_action_input', False)
    if c['randomize_placement_order'] or c['randomize_action_input']:
        c['py_seeds'] = [(c['seed_base'] * 7919 + e) & 0xFFFFFFFF for e in range(c['n_envs'])]
    if 'target_mapping' in c:
        c['target_mapping'] = {f'agent{k}': f'agent{v}' for k, v in c['target_mapping'].items()}
    if c.pop('corners', False):
        corners = [[1, 1], [1, 6], [6, 1], [6, 6]]
        c['initial_positions'] = {i: corners[i % 4] for i in range(c['n_agents'])}
    c['seeds'] = [(c['seed_base'] + e) & 0xFFFFFFFF for e in range(c['n_envs'])]
    c['action_seed'] = 1234 + c['seed_base']
    # json keys must be str
    for k in ('overlap', 'attack_mapping', 'initial_positions', 'initial_health'):
        c[k] = {str(kk): v for kk, v in c[k].items()}
    return c


def make_actions(c, A, managers=None):
    rng = np.random.RandomState(c['action_seed'])
    T, E = c['n_steps'], c['n_envs']
    if c.get('kind') == 'rtt':
        # [move_row, move_col, attack cells ((2R+1)^2, row-major)]
        ra = c['target']['attack_range']
        simul = c['target'].get('simultaneous_attacks', 1)
        D = 2 * ra + 1
        act = np.zeros((T, E, A, 2 + D * D), dtype=np.int8)
        mr = c['runner']['move_range']
        act[..., 0:2] = rng.randint(-mr, mr + 1, size=(T, E, A, 2))
        act[..., 2:] = rng.randint(0, simul + 1, size=(T, E, A, D * D))
        return act
    mr = c['agent']['move_range']
    act = np.zeros((T, E, A, 3), dtype=np.int8)
    act[..., 0:2] = rng.randint(-mr, mr + 1, size=(T, E, A, 2))
    act[..., 2] = rng.randint(0, c.get('attack_max', 1) + 1, size=(T, E, A))
    return act


def build_reference_maze(c):
    from abmarl.examples import MazeNavigationAgent, MazeNavigationSim
    from abmarl.sim.gridworld.agent import GridWorldAgent
    from abmarl.managers import AllStepManager
    registry = {
        'N': lambda n: MazeNavigationAgent(id='navigator', encoding=1,
                                           view_range=c['agent']['view_range']),
        'T': lambda n: GridWorldAgent(id='target', encoding=3),
        'W': lambda n: GridWorldAgent(id=f'wall{n}', encoding=2, blocking=True),
    }
    sim = MazeNavigationSim.build_sim_from_array(
        np.array(c['maze'], dtype=object), registry, overlapping={1: {3}, 3: {1}},
        states={'PositionState'}, observers={'PositionCenteredEncodingObserver'})
    return AllStepManager(sim)


def build_reference_rtt(c):
    from abmarl.examples import ReachTheTargetSim, RunningAgent, TargetAgent, BarrierAgent
    from abmarl.managers import AllStepManager
    R, C = c['rows'], c['cols']
    corners = [[0, 0], [R - 1, 0], [0, C - 1], [R - 1, C - 1]]
    agents = {f'barrier{i}': BarrierAgent(id=f'barrier{i}') for i in range(c['n_barriers'])}
    for i in range(c['n_runners']):
        kw = dict(c['runner'])
        if c.get('corners'):
            kw['initial_position'] = np.array(corners[i % 4], dtype=int)
        agents[f'runner{i}'] = RunningAgent(id=f'runner{i}', **kw)
    kw = dict(c['target'])
    if c.get('corners') or c.get('target_center'):
        kw['initial_position'] = np.array([R // 2, C // 2], dtype=int)
    sim_cls = ReachTheTargetSim
    if 'target_ammo' in c:
        from abmarl.sim.gridworld.agent import AmmoAgent
        from abmarl.sim.gridworld.state import AmmoState

        class AmmoTarget(TargetAgent, AmmoAgent):
            pass

        class AmmoReachTheTargetSim(ReachTheTargetSim):
            def __init__(self, **kwargs):
                super().__init__(**kwargs)
                self.ammo_state = AmmoState(**kwargs)

            def reset(self, **kwargs):
                super().reset(**kwargs)
                self.ammo_state.reset(**kwargs)

        agents['target'] = AmmoTarget(initial_ammo=c['target_ammo'], **kw)
        sim_cls = AmmoReachTheTargetSim
    else:
        agents['target'] = TargetAgent(**kw)
    sim = sim_cls.build_sim(R, C, agents=agents, overlapping={2: {3}, 3: {1, 2, 3}},
                            attack_mapping={2: {3}})
    return AllStepManager(sim, randomize_action_input=c.get('randomize_action_input', False))


def traffic_registry(TrafficAgent, TargetAgent, WallAgent):
    """rllib_traffic_corridor_2_teams.py's object registry."""
    return {
        'R': lambda n: TrafficAgent(id=f'red{n}', encoding=1),
        'G': lambda n: TrafficAgent(id=f'green{n}', encoding=2),
        'r': lambda n: TargetAgent(id='red_target', encoding=1),
        'g': lambda n: TargetAgent(id='green_target', encoding=2),
        'W': lambda n: WallAgent(id=f'wall{n}', encoding=3),
    }


def traffic_mapping(c, ids):
    if c.get('targets') == 'team':
        return {a: ('red_target' if a.startswith('red') and a != 'red_target' else 'green_target')
                for a in ids if a.startswith(('red', 'green')) and not a.endswith('_target')}
    return dict(c['target_mapping'])


def build_reference_traffic(c):
    from abmarl.examples.sim.traffic_corridor import WallAgent, TargetAgent, TrafficAgent, \
        TrafficCorridorSimulation
    from abmarl.managers import AllStepManager
    arr = np.array([list(r) for r in c['grid']], dtype=object)
    reg = traffic_registry(TrafficAgent, TargetAgent, WallAgent)
    probe = TrafficCorridorSimulation.build_sim_from_array(
        arr, reg, overlapping={1: {1}, 2: {2}}, states={'PositionState'},
        observers={'PositionCenteredEncodingObserver'})
    mapping = traffic_mapping(c, list(probe.agents))
    sim = TrafficCorridorSimulation.build_sim_from_array(
        arr, reg, overlapping={1: {1}, 2: {2}}, states={'PositionState'}, dones={'TargetAgentDone'},
        observers={'PositionCenteredEncodingObserver'}, target_mapping=mapping)
    return AllStepManager(sim, randomize_action_input=c.get('randomize_action_input', False))


def len_fixed_team_battle(TeamBattleSim):
    """team_battle_example.py:33-59 with its failed-attack test written as
    len(attacked_agents) == 0 (the example's `not attacked_agents` raises
    ValueError on a numpy array of two or more agents); the step is otherwise
    the example's, statement for statement."""
    class LenFixedTeamBattleSim(TeamBattleSim):
        def step(self, action_dict, **kwargs):
            for agent_id, action in action_dict.items():
                attacking_agent = self.agents[agent_id]
                if attacking_agent.active:
                    status, attacked = self.attack_actor.process_action(attacking_agent, action, **kwargs)
                    if status:
                        if len(attacked) == 0:
                            self.rewards[attacking_agent.id] -= 0.1
                        else:
                            for attacked_agent in attacked:
                                if not attacked_agent.active:
                                    self.rewards[attacked_agent.id] -= 1
                                    self.rewards[attacking_agent.id] += 1
            for agent_id, action in action_dict.items():
                agent = self.agents[agent_id]
                if agent.active:
                    if not self.move_actor.process_action(agent, action, **kwargs):
                        self.rewards[agent.id] -= 0.1
            for agent_id in action_dict:
                self.rewards[agent_id] -= 0.01
    return LenFixedTeamBattleSim


def build_reference_env(c):
    if c['kind'] == 'maze':
        return build_reference_maze(c)
    if c['kind'] == 'traffic':
        return build_reference_traffic(c)
    if c['kind'] == 'rtt':
        return build_reference_rtt(c)
    from abmarl.examples.sim.team_battle_example import TeamBattleSim
    from abmarl.sim.gridworld.agent import GridWorldAgent
    from abmarl.sim.gridworld.agent import GridObservingAgent, MovingAgent, AttackingAgent, \
        HealthAgent
    from abmarl.sim.gridworld.agent import AmmoAgent
    from abmarl.sim.gridworld.state import PositionState, HealthState, AmmoState
    from abmarl.managers import AllStepManager

    class Fighter(GridObservingAgent, MovingAgent, AttackingAgent, HealthAgent):
        pass

    class AmmoFighter(GridObservingAgent, MovingAgent, AttackingAgent, HealthAgent, AmmoAgent):
        pass

    agents = {}
    for i in range(c['n_agents']):
        kw = dict(id=f'agent{i}', encoding=i % c['n_teams'] + 1, **c['agent'])
        if c.get('views'):
            kw['view_range'] = c['views'][i % len(c['views'])]
        if str(i) in c['initial_positions']:
            kw['initial_position'] = np.array(c['initial_positions'][str(i)])
        if str(i) in c['initial_health']:
            kw['initial_health'] = c['initial_health'][str(i)]
        if i in c['blocking']:
            kw['blocking'] = True
        if c.get('ammo'):
            kw['initial_ammo'] = c['ammo'][i % len(c['ammo'])]
            agents[kw['id']] = AmmoFighter(**kw)
        else:
            agents[kw['id']] = Fighter(**kw)
    kwargs = dict(
        overlapping={int(k): set(v) for k, v in c['overlap'].items()},
        attack_mapping={int(k): set(v) for k, v in c['attack_mapping'].items()},
        stacked_attacks=c['stacked_attacks'],
        observe_self=c['observe_self'],
        no_overlap_at_reset=c['no_overlap_at_reset'],
        randomize_placement_order=c.get('randomize_placement_order', False),
        states={'PositionState', 'HealthState'} | ({'AmmoState'} if c.get('ammo') else set()),
        observers={'PositionCenteredEncodingObserver'},
        dones=set(c['dones']))
    if 'target_mapping' in c:
        kwargs['target_mapping'] = dict(c['target_mapping'])
    if c['walls']:
        arr = np.full((c['rows'], c['cols']), '_', dtype=object)
        for r, cc in c['walls']:
            arr[r, cc] = 'W'
        wenc = c['wall_encoding']
        sim = TeamBattleSim.build_sim_from_array(
            arr, {'W': lambda n: GridWorldAgent(id=f'wall{n}', encoding=wenc, blocking=True)},
            extra_agents=agents, **kwargs)
    else:
        sim_cls = TeamBattleSim
        if c.get('len_fix'):
            sim_cls = len_fixed_team_battle(TeamBattleSim)
        sim = sim_cls.build_sim(c['rows'], c['cols'], agents=agents, **kwargs)
    # pin the set-ordered state components (smart.py:37)
    pos = [s for s in sim._states if isinstance(s, PositionState)][0]
    hea = [s for s in sim._states if isinstance(s, HealthState)][0]
    ammo = [s for s in sim._states if isinstance(s, AmmoState)]
    # AmmoState draws nothing: its place in the order changes no result
    sim._states = ([pos, hea] if c['state_order'] == 'position_health' else [hea, pos]) + ammo
    return AllStepManager(sim, randomize_action_input=c.get('randomize_action_input', False))


def run_case(case):
    c = full_case(case)
    T, E = c['n_steps'], c['n_envs']
    S = 2 * c['agent']['view_range'] + 1
    managers = [build_reference_env(c) for _ in range(E)]
    ids = list(managers[0].agents.keys())        # entities, agents-dict order
    A = len(ids)
    act = make_actions(c, A)
    agents0 = list(managers[0].agents.values())

    def obs_array(obs_dict):
        out = np.full((A, S, S), -2, dtype=np.int8)
        ret = np.zeros(A, dtype=np.uint8)
        for i, aid in enumerate(ids):
            if aid in obs_dict:
                o = obs_dict[aid].get('position_centered_encoding')
                if o is not None:           # a window of range v in the top-left of S x S
                    out[i, :o.shape[0], :o.shape[1]] = o
                ret[i] = 1
        return out, ret

    import random
    rng_states, py_states = [], []
    obs0 = np.zeros((E, A, S, S), dtype=np.int8)
    for e in range(E):
        np.random.seed(c['seeds'][e])
        if 'py_seeds' in c:                 # Python's random: randomize_placement_order
            random.seed(c['py_seeds'][e])
        o = managers[e].reset()
        obs0[e], _ = obs_array(o)
        rng_states.append(np.random.get_state())
        py_states.append(random.getstate())

    out = dict(
        obs=np.zeros((T, E, A, S, S), dtype=np.int8),
        returned=np.zeros((T, E, A), dtype=np.uint8),
        reward=np.zeros((T, E, A), dtype=np.float64),
        done=np.ones((T, E, A), dtype=np.uint8),
        all_done=np.zeros((T, E), dtype=np.uint8),
        pos=np.zeros((T, E, A, 2), dtype=np.int8),
        health=np.zeros((T, E, A), dtype=np.float64),
        active=np.zeros((T, E, A), dtype=np.uint8),
        mt_pos=np.zeros((T, E), dtype=np.int16),
        mt_crc=np.zeros((T, E), dtype=np.uint32),
        reset_mask=np.zeros((T, E), dtype=np.uint8),
        err=np.zeros((T, E), dtype=np.uint8),
        reset_obs=np.full((T, E, A, S, S), -2, dtype=np.int8),
        ammo=np.zeros((T, E, A), dtype=np.int16),
    )
    steps = [0] * E
    for t in range(T):
        for e in range(E):
            m = managers[e]
            np.random.set_state(rng_states[e])
            random.setstate(py_states[e])
            adict = {}
            for i, aid in enumerate(ids):
                if aid not in m.done_agents:
                    if c['kind'] == 'rtt':
                        a = {}
                        ag = agents0[i]
                        if hasattr(ag, 'move_range'):
                            a['move'] = act[t, e, i, :2].astype(int)
                        if hasattr(ag, 'attack_range'):
                            d = 2 * ag.attack_range + 1
                            a['attack'] = act[t, e, i, 2:2 + d * d].astype(int).reshape(d, d)
                        adict[aid] = a
                    elif c['kind'] == 'traffic':
                        adict[aid] = {'move': act[t, e, i, :2].astype(int)}
                    else:
                        adict[aid] = {'move': act[t, e, i, :2].astype(int),
                                      'attack': int(act[t, e, i, 2])}
            try:
                o, r, d, _ = m.step(adict)
            except (KeyError, ValueError) as ex:
                # KeyError (err 1): reach_the_target.py:118-120, Grid.remove of a
                # runner the target already killed on its cell; ValueError (err
                # 2): `not attacked_agents` on BinaryAttackActor's numpy array
                # (team_battle_example.py:41).  The env must be reset.
                out['err'][t, e] = 1 if isinstance(ex, KeyError) else 2
                steps[e] = c['horizon']
                out['mt_pos'][t, e] = np.random.get_state()[2]
                out['mt_crc'][t, e] = zlib.crc32(np.ascontiguousarray(np.random.get_state()[1],
                                                                      dtype=np.uint32).tobytes())
                ro = m.reset()
                steps[e] = 0
                out['reset_mask'][t, e] = 1
                out['reset_obs'][t, e], _ = obs_array(ro)
                rng_states[e] = np.random.get_state()
                py_states[e] = random.getstate()
                continue
            steps[e] += 1
            out['obs'][t, e], out['returned'][t, e] = obs_array(o)
            for i, aid in enumerate(ids):
                if aid in r:
                    out['reward'][t, e, i] = r[aid]
                    out['done'][t, e, i] = int(bool(d[aid]))
                agent = m.agents[aid]
                out['pos'][t, e, i] = agent.position
                out['health'][t, e, i] = getattr(agent, 'health', 0.0)
                out['active'][t, e, i] = int(agent.active)
                out['ammo'][t, e, i] = getattr(agent, 'ammo', 0)
            out['all_done'][t, e] = int(bool(d['__all__']))
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
    print(f"{c['name']}: {T} steps x {E} envs x {A} entities, resets={int(out['reset_mask'].sum())}, "
          f"kills/arrivals={int((out['reward'] > 0.5).sum())} -> {os.path.getsize(path)} B")


def run_multicorridor(randomize=False, n_steps=60):
    """BASELINE config 1: MultiCorridor + AllStepManager, np.random.seed(24)
    (tests/test_all_step_multi_corridor.py), scripted random actions."""
    import random
    from abmarl.examples import MultiCorridor
    from abmarl.managers import AllStepManager
    rng = np.random.RandomState(99)
    np.random.seed(24)
    random.seed(24)
    sim = AllStepManager(MultiCorridor(), randomize_action_input=randomize)

    def enc(d):
        return {k: {kk: np.asarray(vv).tolist() for kk, vv in v.items()} for k, v in d.items()}

    records = [{'reset': enc(sim.reset())}]
    for t in range(n_steps):
        acts = {aid: int(rng.randint(0, 3)) for aid in sim.agents if aid not in sim.done_agents}
        o, r, d, _ = sim.step(acts)
        rec = {'actions': acts, 'obs': enc(o), 'reward': {k: float(v) for k, v in r.items()},
               'done': {k: bool(v) for k, v in d.items()}}
        if d['__all__']:
            rec['reset'] = enc(sim.reset())
        records.append(rec)
    name = 'multicorridor_shuffled' if randomize else 'multicorridor'
    path = os.path.join(HERE, name + '.json')
    json.dump(records, open(path, 'w'))
    print(f"{name}: {n_steps} steps -> {os.path.getsize(path)} B")


def run_multicorridor_turn_based(n_steps=300):
    """TurnBasedManager over MultiCorridor, np.random.seed(24)
    (tests/test_turn_based_multi_corridor.py), scripted random actions for the
    agent whose turn it is; the cycle is NOT restarted by reset (the
    reference's agent_order is created once, turn_based_manager.py:17-20)."""
    from abmarl.examples import MultiCorridor
    from abmarl.managers import TurnBasedManager
    rng = np.random.RandomState(7)
    np.random.seed(24)
    sim = TurnBasedManager(MultiCorridor())

    def enc(d):
        return {k: {kk: np.asarray(vv).tolist() for kk, vv in v.items()} for k, v in d.items()}

    o = sim.reset()
    records = [{'reset': enc(o)}]
    for t in range(n_steps):
        actor = [k for k in o if k not in sim.done_agents][-1]
        acts = {actor: int(rng.choice(3, p=[0.2, 0.2, 0.6]))}   # mostly RIGHT
        o, r, d, _ = sim.step(acts)
        rec = {'actions': acts, 'obs': enc(o), 'reward': {k: float(v) for k, v in r.items()},
               'done': {k: bool(v) for k, v in d.items()}}
        if d['__all__']:
            o = sim.reset()
            rec['reset'] = enc(o)
        records.append(rec)
    path = os.path.join(HERE, 'multicorridor_turn.json')
    json.dump(records, open(path, 'w'))
    print(f"multicorridor_turn: {n_steps} steps -> {os.path.getsize(path)} B")


def main():
    sys.path.insert(0, HERE)
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    only = sys.argv[1:]
    if 'multicorridor_turn' in only:
        run_multicorridor_turn_based()
    for case in CASES:
        if not only or case['name'] in only:
            run_case(case)
    if only:
        return
    run_multicorridor(False)
    run_multicorridor(True)
    run_multicorridor_turn_based()


if __name__ == '__main__':
    main()
