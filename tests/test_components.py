"""The component plugin API on the device (gw_component, component_runtime.py).

Two kinds of evidence:
  * the reference's own component unit tests (tests/sim/gridworld/
    test_state.py, test_actor.py, test_observer.py in the reference) restated
    with their scenarios and known answers, every component call running as
    a gw_component operation on the GPU;
  * a user-written simulation -- the reference's TeamBattle example step()
    (examples/sim/team_battle_example.py:33-59) written here against the
    components, with no engine program -- driven by AllStepManager through
    the reference's golden trajectories (tests/golden/*.npz), bit-exact in
    observations, float64 rewards, dones, positions, health, active flags
    and the numpy MT19937 state after every step.

CPU tests at the bottom cover construction-time validation and that the
runtime refuses to run without the HIP engine.
"""
import zlib

import numpy as np
import pytest

from abmarl_amd.sim.gridworld.grid import Grid
from abmarl_amd.sim.gridworld.agent import (
    GridWorldAgent, GridObservingAgent, MovingAgent, AttackingAgent, HealthAgent, AmmoAgent)
from abmarl_amd.sim.gridworld.components import (
    PositionState, HealthState, AmmoState, MoveActor, BinaryAttackActor, SelectiveAttackActor,
    PositionCenteredEncodingObserver)
from abmarl_amd.sim.gridworld.smart import SmartGridWorldSimulation
from abmarl_amd.managers import AllStepManager

gpu = pytest.mark.gpu
KEY = 'position_centered_encoding'


@pytest.fixture(params=['wave', 'workgroup'], autouse=True)
def component_kernel(request):
    """Every GPU test of this module on both component kernels: the one-wave
    comp_kernel and the workgroup-per-env wg_comp_kernel (forced below its
    usual > 64-entity threshold)."""
    from abmarl_amd.sim.gridworld.component_runtime import ComponentRuntime
    if request.param == 'workgroup':
        if request.node.get_closest_marker('gpu') is None:
            pytest.skip('CPU test: one kernel')
        if 'tb_views' in request.node.name or 'position_centered_observer' in request.node.name or \
                'observe_self' in request.node.name:
            pytest.skip('observers with different view ranges: the one-wave kernel only')
        if 'randomize_placement_order' in request.node.name or 'tb_order' in request.node.name:
            pytest.skip('randomize_placement_order / placement orders: the one-wave kernel only')
    ComponentRuntime.force_workgroup = request.param == 'workgroup'
    yield request.param
    ComponentRuntime.force_workgroup = False


# ------------------------------------------------------------------ states
@gpu
def test_position_state_randomize_placement_order():
    """state.py:97-101: random.shuffle of the agents dict before every
    placement; known answers from the reference itself
    (tests/golden/make_shuffle_known_answers.py: six resets after
    random.seed(3), np.random.seed(5)), cell insertion order included, and
    both RNG streams left where the reference leaves them."""
    import random
    agents = {'a0': GridWorldAgent(id='a0', encoding=1), 'a1': GridWorldAgent(id='a1', encoding=2),
              'a2': GridWorldAgent(id='a2', encoding=1, initial_position=np.array([0, 0])),
              'a3': GridWorldAgent(id='a3', encoding=2), 'a4': GridWorldAgent(id='a4', encoding=1)}
    grid = Grid(2, 3, overlapping={1: {1}})
    state = PositionState(grid=grid, agents=agents, randomize_placement_order=True)
    ref = [[[1, 0], [0, 2], [0, 0], [1, 1], [0, 0], ['a2', 'a4']],
           [[1, 0], [0, 1], [0, 0], [1, 2], [0, 0], ['a2', 'a4']],
           [[0, 1], [1, 2], [0, 0], [1, 1], [0, 0], ['a2', 'a4']],
           [[0, 0], [1, 1], [0, 0], [0, 1], [1, 2], ['a2', 'a0']],
           [[1, 2], [1, 1], [0, 0], [0, 2], [0, 1], ['a2']],
           [[0, 1], [1, 0], [0, 0], [1, 2], [0, 1], ['a2']]]
    random.seed(3)
    np.random.seed(5)
    for k, want in enumerate(ref):
        state.reset()
        got = [list(map(int, agents[a].position)) for a in ['a0', 'a1', 'a2', 'a3', 'a4']]
        assert got == want[:5], (k, got, want)
        assert list(grid[0, 0]) == want[5], (k, list(grid[0, 0]))
    assert np.random.get_state()[2] == 38
    assert random.random() == 0.6714114753695926


@gpu
def test_position_state_initial_positions():
    """test_state.py:11-28."""
    grid = Grid(3, 3)
    agents = {f'agent{i}': GridWorldAgent(id=f'agent{i}', encoding=1, initial_position=np.array(p))
              for i, p in enumerate([(0, 1), (1, 2), (2, 0)])}
    PositionState(grid=grid, agents=agents).reset()
    for aid, p in zip(agents, [(0, 1), (1, 2), (2, 0)]):
        np.testing.assert_equal(agents[aid].position, np.array(p))
        assert grid[p] == {aid: agents[aid]}


@gpu
def test_position_state_no_overlap_at_reset():
    """test_state.py:31-56: initial positions may overlap, drawn ones may not."""
    grid = Grid(3, 3, overlapping={1: {1}})
    init = {3: (2, 2), 8: (0, 0), 9: (0, 0)}
    agents = {}
    for i in range(10):
        kw = dict(initial_position=np.array(init[i])) if i in init else {}
        agents[f'agent{i}'] = GridWorldAgent(id=f'agent{i}', encoding=1, **kw)
    PositionState(grid=grid, agents=agents, no_overlap_at_reset=True).reset()
    assert grid[0, 0] == {'agent8': agents['agent8'], 'agent9': agents['agent9']}
    assert grid[2, 2] == {'agent3': agents['agent3']}
    for cell in [(0, 1), (0, 2), (1, 0), (1, 1), (1, 2), (2, 0), (2, 1)]:
        assert len(grid[cell]) == 1


@gpu
def test_position_state_small_grid():
    """test_state.py:59-110, including the seed-24 pass / seed-17 failure."""
    grid = Grid(1, 2, overlapping={1: {1, 2}, 2: {1, 2}, 3: {3}})
    spec = [(1, (0, 0)), (2, (0, 0)), (3, None), (3, None), (2, None), (1, None)]
    agents = {f'agent{i}': GridWorldAgent(
        id=f'agent{i}', encoding=e, **({} if p is None else dict(initial_position=np.array(p))))
        for i, (e, p) in enumerate(spec)}
    PositionState(grid=grid, agents=agents).reset()
    for aid, cell in [('agent0', (0, 0)), ('agent1', (0, 0)), ('agent2', (0, 1)),
                      ('agent3', (0, 1)), ('agent4', (0, 0)), ('agent5', (0, 0))]:
        assert aid in grid[cell]

    agents = {'agent0': GridWorldAgent(id='agent0', encoding=1, initial_position=np.array([0, 0])),
              'agent1': GridWorldAgent(id='agent1', encoding=2, initial_position=np.array([0, 1])),
              'agent2': GridWorldAgent(id='agent2', encoding=3)}
    with pytest.raises(RuntimeError):
        PositionState(grid=grid, agents=agents).reset()

    np.random.seed(24)
    agents = {'agent0': GridWorldAgent(id='agent0', encoding=1, initial_position=np.array([0, 0])),
              'agent1': GridWorldAgent(id='agent1', encoding=2),
              'agent2': GridWorldAgent(id='agent2', encoding=3)}
    ps = PositionState(grid=grid, agents=agents)
    ps.reset()
    assert 'agent0' in grid[0, 0] and 'agent1' in grid[0, 0] and 'agent2' in grid[0, 1]
    np.random.seed(17)
    with pytest.raises(RuntimeError):
        ps.reset()


@gpu
def test_health_state():
    """test_state.py:113-130 (initial health kept exactly, others uniform(0, 1))."""
    grid = Grid(3, 3)
    agents = {'agent0': HealthAgent(id='agent0', encoding=1, initial_health=0.24),
              'agent1': HealthAgent(id='agent1', encoding=1),
              'agent2': HealthAgent(id='agent2', encoding=1)}
    np.random.seed(5)
    HealthState(agents=agents, grid=grid).reset()
    assert agents['agent0'].health == 0.24
    # the two draws are numpy's uniform(0, 1) in agents order
    np.random.seed(5)
    expect = np.random.uniform(0, 1, 2)
    assert [agents['agent1'].health, agents['agent2'].health] == list(expect)
    assert all(a.active for a in agents.values())


# ------------------------------------------------------------------ actors
@gpu
def test_move_actor():
    """test_actor.py:22-78."""
    grid = Grid(5, 6)
    spec = [((3, 4), 1, 1), ((2, 2), 2, 2), ((0, 1), 1, 1), ((3, 1), 3, 3)]
    agents = {f'agent{i}': MovingAgent(id=f'agent{i}', initial_position=np.array(p), encoding=e,
                                       move_range=r) for i, (p, e, r) in enumerate(spec)}
    ps = PositionState(grid=grid, agents=agents)
    move = MoveActor(grid=grid, agents=agents)
    ps.reset()
    for moves in ([(1, 1), (-1, 0), (0, 1), (-1, 1)], [(1, 1), (0, 0), (-1, 1), (-1, 0)]):
        for aid, m in zip(agents, moves):
            move.process_action(agents[aid], {'move': np.array(m)})
        for aid, p in zip(agents, [(4, 5), (1, 2), (0, 2), (2, 2)]):
            np.testing.assert_array_equal(agents[aid].position, np.array(p))


@gpu
def test_move_actor_with_overlap():
    """test_actor.py:81-131."""
    grid = Grid(5, 6, overlapping={1: {1}, 2: {3}, 3: {2}})
    spec = [((4, 4), 1, 1), ((2, 2), 2, 2), ((2, 4), 1, 1), ((3, 2), 3, 3)]
    agents = {f'agent{i}': MovingAgent(id=f'agent{i}', initial_position=np.array(p), encoding=e,
                                       move_range=r) for i, (p, e, r) in enumerate(spec)}
    ps = PositionState(grid=grid, agents=agents)
    move = MoveActor(grid=grid, agents=agents)
    ps.reset()
    rounds = [([(-1, 0), (0, 0), (1, 0), (-1, 0)], [(3, 4), (2, 2), (3, 4), (2, 2)]),
              ([(-1, 0), (0, 2), (0, -1), (1, 1)], [(2, 4), (2, 2), (3, 3), (2, 2)])]
    for moves, expect in rounds:
        for aid, m in zip(agents, moves):
            move.process_action(agents[aid], {'move': np.array(m)})
        for aid, p in zip(agents, expect):
            np.testing.assert_array_equal(agents[aid].position, np.array(p))
    # the grid container follows the engine: two agents share (2, 2)
    assert set(grid[2, 2]) == {'agent1', 'agent3'}


@gpu
def test_static_wall_edited_on_the_host():
    """A wall (a static entity: the engine keeps it in its cell template) that
    the host removes through Grid.remove stops blocking, and one the host
    places elsewhere blocks there: the runtime sees the edit and rebuilds
    with every entity a lane (reference semantics: Grid.query on the host's
    cells, grid.py:81-140)."""
    grid = Grid(3, 3)
    agents = {'mover': MovingAgent(id='mover', initial_position=np.array([1, 0]), encoding=1, move_range=1),
              'wall': GridWorldAgent(id='wall', initial_position=np.array([1, 1]), encoding=3)}
    ps = PositionState(grid=grid, agents=agents)
    move = MoveActor(grid=grid, agents=agents)
    ps.reset()
    mover, wall = agents['mover'], agents['wall']
    assert not move.process_action(mover, {'move': np.array([0, 1])})     # the wall blocks
    np.testing.assert_array_equal(mover.position, [1, 0])
    grid.remove(wall, (1, 1))
    assert move.process_action(mover, {'move': np.array([0, 1])})         # now the cell is empty
    np.testing.assert_array_equal(mover.position, [1, 1])
    assert grid.place(wall, (1, 2))
    assert not move.process_action(mover, {'move': np.array([0, 1])})     # blocked at its new cell
    np.testing.assert_array_equal(mover.position, [1, 1])
    assert move.process_action(mover, {'move': np.array([-1, 0])})
    np.testing.assert_array_equal(mover.position, [0, 1])
    assert set(grid[1, 2]) == {'wall'} and not grid[1, 1]


@gpu
def test_in_place_host_edit_is_seen():
    """Edits that bump no host version -- an element of an agent's position
    array and the Grid's cell dicts written directly -- still reach the
    device before the next component call (the runtime's fingerprint)."""
    grid = Grid(4, 4)
    agents = {'mover': MovingAgent(id='mover', initial_position=np.array([1, 0]), encoding=1, move_range=1)}
    ps = PositionState(grid=grid, agents=agents)
    move = MoveActor(grid=grid, agents=agents)
    ps.reset()
    mover = agents['mover']
    assert move.process_action(mover, {'move': np.array([1, 0])})
    np.testing.assert_array_equal(mover.position, [2, 0])
    del grid[2, 0]['mover']
    grid[2, 2]['mover'] = mover
    mover.position[1] = 2                                               # in place: (2, 2)
    assert move.process_action(mover, {'move': np.array([-1, 0])})
    np.testing.assert_array_equal(mover.position, [1, 2])
    assert set(grid[1, 2]) == {'mover'} and not grid[2, 2] and not grid[2, 0]


def _attack_agents(attacker_kw, health=None):
    h = {} if health is None else dict(initial_health=health)
    return {
        'agent0': HealthAgent(id='agent0', initial_position=np.array([4, 4]), encoding=1, **h),
        'agent1': AttackingAgent(id='agent1', initial_position=np.array([2, 2]), encoding=1,
                                 attack_range=2, **attacker_kw),
        'agent2': HealthAgent(id='agent2', initial_position=np.array([2, 3]), encoding=2, **h),
        'agent3': HealthAgent(id='agent3', initial_position=np.array([3, 2]), encoding=1, **h),
    }


@gpu
def test_binary_attack_actor():
    """test_actor.py:454-500."""
    grid = Grid(5, 6)
    agents = _attack_agents(dict(attack_strength=1, attack_accuracy=1))
    ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
    attack = BinaryAttackActor(attack_mapping={1: {1}}, grid=grid, agents=agents)
    ps.reset()
    hs.reset()
    for _ in range(2):
        status, attacked = attack.process_action(agents['agent1'], {'attack': 1})
        assert status and attacked
    assert not agents['agent0'].active and not agents['agent3'].active
    assert agents['agent0'].health <= 0 and agents['agent3'].health <= 0
    assert not grid[4, 4] and not grid[3, 2]
    status, attacked = attack.process_action(agents['agent1'], {'attack': 1})
    assert status and not attacked
    assert agents['agent2'].active and agents['agent2'].health > 0 and grid[2, 3]


@gpu
def test_binary_attack_actor_simultaneous_attacks():
    """test_actor.py:531-591 (attack_strength changed between calls)."""
    grid = Grid(5, 6)
    agents = {
        'agent0': AttackingAgent(id='agent0', initial_position=np.array([2, 2]), encoding=1,
                                 attack_range=2, attack_strength=0, attack_accuracy=1,
                                 simultaneous_attacks=3),
        'agent1': HealthAgent(id='agent1', initial_position=np.array([4, 4]), encoding=1,
                              initial_health=1),
        'agent2': HealthAgent(id='agent2', initial_position=np.array([2, 3]), encoding=2,
                              initial_health=1),
        'agent3': HealthAgent(id='agent3', initial_position=np.array([3, 2]), encoding=1,
                              initial_health=1),
    }
    ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
    attack = BinaryAttackActor(attack_mapping={1: {1, 2}}, grid=grid, agents=agents)
    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent0'], {'attack': 0})
    assert not status and not attacked
    for n in (1, 2, 3):
        status, attacked = attack.process_action(agents['agent0'], {'attack': n})
        assert status and len(attacked) == n
    agents['agent0'].attack_strength = 1
    status, attacked = attack.process_action(agents['agent0'], {'attack': 3})
    assert status and len(attacked) == 3
    for aid in ('agent1', 'agent2', 'agent3'):
        assert not agents[aid].active and agents[aid].health <= 0
    assert not grid[4, 4] and not grid[2, 3] and not grid[3, 2]


@gpu
def test_binary_attack_actor_stacked_attack():
    """test_actor.py:649-721: two actors with different mappings / stacking on one grid."""
    grid = Grid(5, 6)
    agents = {
        'agent0': AttackingAgent(id='agent0', initial_position=np.array([2, 2]), encoding=1,
                                 attack_range=2, attack_strength=1, attack_accuracy=1,
                                 simultaneous_attacks=2),
        'agent1': HealthAgent(id='agent1', initial_position=np.array([4, 4]), encoding=1,
                              initial_health=1),
        'agent2': HealthAgent(id='agent2', initial_position=np.array([2, 3]), encoding=2,
                              initial_health=1),
        'agent3': HealthAgent(id='agent3', initial_position=np.array([3, 2]), encoding=1,
                              initial_health=1),
    }
    ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
    attack = BinaryAttackActor(attack_mapping={1: {1}}, stacked_attacks=False, grid=grid,
                               agents=agents)
    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent0'], {'attack': 2})
    assert status and len(attacked) == 2
    assert agents['agent1'] in attacked and agents['agent3'] in attacked
    assert agents['agent2'] not in attacked
    assert not agents['agent1'].active and not agents['agent3'].active
    assert not grid[4, 4] and not grid[3, 2]

    agents['agent0'].attack_strength = 0.5
    attack = BinaryAttackActor(attack_mapping={1: {2}}, stacked_attacks=True, grid=grid,
                               agents=agents)
    status, attacked = attack.process_action(agents['agent0'], {'attack': 1})
    assert status and attacked == [agents['agent2']]
    assert agents['agent2'].health == 0.5
    agents['agent0'].attack_strength = 0
    status, attacked = attack.process_action(agents['agent0'], {'attack': 2})
    assert status and len(attacked) == 2 and attacked[0] == attacked[1]
    assert agents['agent2'].health == 0.5
    agents['agent0'].attack_strength = 0.25
    status, attacked = attack.process_action(agents['agent0'], {'attack': 2})
    assert status and len(attacked) == 2 and attacked[0] == attacked[1]
    assert not agents['agent2'].active and agents['agent2'].health <= 0
    assert not grid[2, 3]


def _cells(*hits, fill=0):
    a = np.full((5, 5), fill, dtype=int)
    for r, c in hits:
        a[r, c] = 1 - fill
    return {'attack': a}


@gpu
def test_selective_attack_actor():
    """test_actor.py:724-882 (attacked lists in the reference's cell order)."""
    grid = Grid(5, 6)
    agents = _attack_agents(dict(attack_strength=1, attack_accuracy=1))
    ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
    attack = SelectiveAttackActor(attack_mapping={1: {1}}, grid=grid, agents=agents)
    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent1'], _cells((4, 4)))
    assert status and attacked == [agents['agent0']]
    assert not agents['agent0'].active and agents['agent0'].health <= 0 and not grid[4, 4]
    status, attacked = attack.process_action(agents['agent1'], _cells((3, 2)))
    assert status and attacked == [agents['agent3']]
    assert not agents['agent3'].active and not grid[3, 2]

    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent1'], _cells((3, 2), (4, 4)))
    assert status and attacked == [agents['agent3'], agents['agent0']]
    assert not grid[4, 4] and not grid[3, 2]

    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent1'], _cells((3, 2), (4, 4), fill=1))
    assert status and not attacked
    assert all(a.active for a in agents.values())
    assert grid[4, 4] and grid[3, 2] and grid[2, 2] and grid[2, 3]
    status, attacked = attack.process_action(agents['agent1'], _cells(fill=1))
    assert status and attacked == [agents['agent3'], agents['agent0']]
    assert agents['agent1'].active and agents['agent2'].active
    assert not grid[4, 4] and not grid[3, 2] and grid[2, 2] and grid[2, 3]

    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent1'], _cells())
    assert not status and not attacked
    assert all(a.active for a in agents.values())


class AttackerWithAmmo(AttackingAgent, AmmoAgent):
    pass


@gpu
def test_binary_attack_actor_ammo():
    """test_actor.py:594-646: an AmmoAgent with 5 rounds attacks once, twice,
    then three times with two targets in reach: the ammo filter
    (actor.py:343-351) keeps 2 of the last attack's picks."""
    grid = Grid(5, 6)
    agents = {
        'agent0': AttackerWithAmmo(id='agent0', initial_position=np.array([2, 2]), encoding=1,
                                   attack_range=2, attack_strength=0, attack_accuracy=1,
                                   simultaneous_attacks=3, initial_ammo=5),
        'agent1': HealthAgent(id='agent1', initial_position=np.array([4, 4]), encoding=1, initial_health=1),
        'agent2': HealthAgent(id='agent2', initial_position=np.array([2, 3]), encoding=2, initial_health=1),
        'agent3': HealthAgent(id='agent3', initial_position=np.array([3, 2]), encoding=1, initial_health=1),
    }
    ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
    ammo_state = AmmoState(grid=grid, agents=agents)
    attack = BinaryAttackActor(attack_mapping={1: {1, 2}}, grid=grid, agents=agents)
    from abmarl_amd.spaces import Discrete
    assert agents['agent0'].action_space['attack'] == Discrete(4)
    ps.reset()
    hs.reset()
    ammo_state.reset()
    status, attacked = attack.process_action(agents['agent0'], {'attack': 0})
    assert not status and not attacked
    status, attacked = attack.process_action(agents['agent0'], {'attack': 1})
    assert status and len(attacked) == 1 and agents['agent0'].ammo == 4
    status, attacked = attack.process_action(agents['agent0'], {'attack': 2})
    assert status and len(attacked) == 2 and agents['agent0'].ammo == 2
    status, attacked = attack.process_action(agents['agent0'], {'attack': 3})
    assert status and len(attacked) == 2 and agents['agent0'].ammo == 0


@gpu
def test_selective_attack_actor_ammo():
    """test_actor.py:885-985: a SelectiveAttackActor attacker with 3 rounds;
    the two-cell attack at 1 round keeps one victim, the whole-window attack
    at 0 rounds none."""
    grid = Grid(5, 6)
    agents = {
        'agent0': HealthAgent(id='agent0', initial_position=np.array([4, 4]), encoding=1),
        'agent1': AttackerWithAmmo(id='agent1', initial_position=np.array([2, 2]), encoding=1,
                                   attack_range=2, attack_strength=1, attack_accuracy=1, initial_ammo=3),
        'agent2': HealthAgent(id='agent2', initial_position=np.array([2, 3]), encoding=2),
        'agent3': HealthAgent(id='agent3', initial_position=np.array([3, 2]), encoding=1),
    }
    ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
    ammo_state = AmmoState(grid=grid, agents=agents)
    attack = SelectiveAttackActor(attack_mapping={1: {1}}, grid=grid, agents=agents)
    ps.reset()
    hs.reset()
    ammo_state.reset()
    status, attacked = attack.process_action(agents['agent1'], _cells((4, 4)))
    assert status and attacked == [agents['agent0']]
    assert not agents['agent0'].active and agents['agent0'].health <= 0 and not grid[4, 4]
    assert agents['agent1'].ammo == 2
    status, attacked = attack.process_action(agents['agent1'], _cells((3, 2)))
    assert status and attacked == [agents['agent3']]
    assert not agents['agent3'].active and agents['agent3'].health <= 0 and not grid[3, 2]
    assert agents['agent1'].ammo == 1

    ps.reset()
    hs.reset()
    status, attacked = attack.process_action(agents['agent1'], _cells((3, 2), (4, 4)))
    assert status and len(attacked) == 1
    assert agents['agent1'].ammo == 0

    status, attacked = attack.process_action(agents['agent1'], _cells(fill=1))
    assert status and not attacked
    assert agents['agent1'].ammo == 0


@gpu
def test_ammo_filter_draws_like_numpy():
    """The filter's draws: an AmmoAgent at 1 round attacking 3 targets keeps
    np.random.choice(attacked, 1, replace=False)[0] of the (cell, insertion)
    ordered candidates -- computed here with numpy itself from the same seed
    -- and leaves np.random where numpy's choice leaves it."""
    for seed in range(6):
        grid = Grid(3, 3)
        agents = {'a': AttackerWithAmmo(id='a', initial_position=np.array([1, 1]), encoding=1,
                                        attack_range=1, attack_strength=1, attack_accuracy=1,
                                        simultaneous_attacks=3, initial_ammo=1)}
        for k, p in enumerate([(0, 0), (0, 2), (2, 1)]):
            agents[f'v{k}'] = HealthAgent(id=f'v{k}', initial_position=np.array(p), encoding=2,
                                          initial_health=1)
        ps, hs = PositionState(grid=grid, agents=agents), HealthState(grid=grid, agents=agents)
        ammo_state = AmmoState(grid=grid, agents=agents)
        attack = BinaryAttackActor(attack_mapping={1: {2}}, grid=grid, agents=agents)
        ps.reset()
        hs.reset()
        ammo_state.reset()
        np.random.seed(seed)
        ref = np.random.RandomState(seed)
        for _ in range(3):                    # _basic_criteria: one uniform() per candidate
            ref.uniform()
        cands = [agents['v0'], agents['v1'], agents['v2']]
        picks = ref.choice(np.array(cands, dtype=object), size=3, replace=False)   # _subset_attackables
        kept = ref.choice(picks, size=1, replace=False).tolist()                  # the ammo filter
        status, attacked = attack.process_action(agents['a'], {'attack': 3})
        assert status and attacked == kept, seed
        assert agents['a'].ammo == 0
        assert np.random.get_state()[2] == ref.get_state()[2]
        assert not kept[0].active and all(v.active for v in cands if v is not kept[0])


# --------------------------------------------------------------- observers
def _observer_agents(blocking):
    return {
        'agent0': GridObservingAgent(id='agent0', encoding=1, view_range=2,
                                     initial_position=np.array([2, 2])),
        'agent1': GridObservingAgent(id='agent1', encoding=2, view_range=1,
                                     initial_position=np.array([0, 0])),
        'agent2': GridObservingAgent(id='agent2', encoding=3, view_range=4,
                                     initial_position=np.array([4, 4])),
        'agent3': GridWorldAgent(id='agent3', encoding=5, initial_position=np.array([3, 3]),
                                 blocking=blocking),
        'agent4': GridWorldAgent(id='agent4', encoding=4, initial_position=np.array([1, 1]),
                                 blocking=blocking),
        'agent5': GridWorldAgent(id='agent5', encoding=6, initial_position=np.array([2, 1]),
                                 blocking=blocking),
    }


N = -1
OUT9 = [[N] * 9] * 4


@gpu
@pytest.mark.parametrize('blocking', [False, True])
def test_position_centered_observer(blocking):
    """test_observer.py:194-339: views 2, 1 and 4 on one grid, with and
    without blocking walls."""
    grid = Grid(5, 5)
    agents = _observer_agents(blocking)
    ps = PositionState(grid=grid, agents=agents)
    observer = PositionCenteredEncodingObserver(agents=agents, grid=grid)
    ps.reset()
    if not blocking:
        e0 = [[2, 0, 0, 0, 0], [0, 4, 0, 0, 0], [0, 6, 1, 0, 0], [0, 0, 0, 5, 0], [0, 0, 0, 0, 3]]
        e2 = [r + [N] * 4 for r in e0] + OUT9
    else:
        e0 = [[-2, -2, 0, 0, 0], [-2, 4, 0, 0, 0], [-2, 6, 1, 0, 0], [-2, 0, 0, 5, -2],
              [0, 0, 0, -2, -2]]
        e2 = [r + [N] * 4 for r in [[-2, -2, -2, 0, 0], [-2, -2, -2, 0, 0], [-2, -2, -2, -2, 0],
                                    [0, 0, -2, 5, 0], [0, 0, 0, 0, 3]]] + OUT9
    e1 = [[N, N, N], [N, 2, 0], [N, 0, 4]]
    for aid, expect in (('agent0', e0), ('agent1', e1), ('agent2', e2)):
        np.testing.assert_array_equal(observer.get_obs(agents[aid])[KEY], np.array(expect))
    assert observer.get_obs(agents['agent3']) == {}


@gpu
def test_observe_self():
    """test_observer.py:844-903: two observers (observe_self True / False)
    sharing one grid, seed 24, two agents on one cell."""
    np.random.seed(24)

    class HackAgent(GridObservingAgent, MovingAgent):
        pass

    agents = {
        'agent0': GridObservingAgent(id='agent0', encoding=1, view_range=2,
                                     initial_position=np.array([2, 2])),
        'agent1': GridObservingAgent(id='agent1', encoding=2, view_range=1,
                                     initial_position=np.array([0, 0])),
        'agent2': HackAgent(id='agent2', encoding=2, view_range=1,
                            initial_position=np.array([2, 2]), move_range=1),
    }
    grid = Grid(5, 5, overlapping={1: {2}, 2: {1}})
    PositionState(grid=grid, agents=agents).reset()
    self_obs = PositionCenteredEncodingObserver(agents=agents, grid=grid)
    no_self = PositionCenteredEncodingObserver(agents=agents, grid=grid, observe_self=False)
    z5 = np.zeros((5, 5), int)
    e = z5.copy(); e[0, 0] = 2; e[2, 2] = 1
    np.testing.assert_array_equal(self_obs.get_obs(agents['agent0'])[KEY], e)
    e[2, 2] = 2
    np.testing.assert_array_equal(no_self.get_obs(agents['agent0'])[KEY], e)
    np.testing.assert_array_equal(self_obs.get_obs(agents['agent1'])[KEY],
                                  np.array([[N, N, N], [N, 2, 0], [N, 0, 0]]))
    np.testing.assert_array_equal(no_self.get_obs(agents['agent1'])[KEY],
                                  np.array([[N, N, N], [N, 0, 0], [N, 0, 0]]))


# ------------------------------------------- a user-written step() on the API
class UserTeamBattle(SmartGridWorldSimulation):
    """The reference's TeamBattle example (team_battle_example.py:23-59) as a
    user would write it: no engine program, its step() composed from the
    components; every component call is a device operation."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.move_actor = MoveActor(**kwargs)
        self.attack_actor = BinaryAttackActor(**kwargs)
        self.finalize()

    # the len_fix fixtures (tb_ammo_multi, tb_ammo_stacked) ran the example
    # with `len(attacked) == 0` as its failed-attack test; the reference's
    # `not attacked` raises ValueError on BinaryAttackActor's numpy array of
    # 2 or more agents, which the component API returns as such
    len_fix = False

    def step(self, action_dict, **kwargs):
        for agent_id, action in action_dict.items():
            agent = self.agents[agent_id]
            if agent.active:
                status, attacked = self.attack_actor.process_action(agent, action, **kwargs)
                if status:
                    if (len(attacked) == 0) if self.len_fix else not attacked:
                        self.rewards[agent_id] -= 0.1
                    else:
                        for other in attacked:
                            if not other.active:
                                self.rewards[other.id] -= 1
                                self.rewards[agent_id] += 1
        for agent_id, action in action_dict.items():
            agent = self.agents[agent_id]
            if agent.active:
                if not self.move_actor.process_action(agent, action, **kwargs):
                    self.rewards[agent.id] -= 0.1
        for agent_id in action_dict:
            self.rewards[agent_id] -= 0.01


def _obs_array(obs, ids, S):
    out = np.full((len(ids), S, S), -2, dtype=np.int64)
    for i, aid in enumerate(ids):
        o = obs.get(aid, {}).get(KEY)
        if o is not None:
            out[i, :o.shape[0], :o.shape[1]] = o
    return out


USER_CASES = [('tb_small', 40, 3), ('tb_order', 30, 2), ('tb_walls', 30, 2),
              ('tb_destroy', 30, 2), ('tb_chase', 30, 2), ('tb_views', 25, 2),
              ('tb_ammo', 50, 2), ('tb_ammo_multi', 50, 2), ('tb_value_error', 60, 3),
              ('tb_value_error_ammo', 40, 2), ('tb_ammo_negative', 40, 2)]


@gpu
@pytest.mark.parametrize('name,steps,envs', USER_CASES)
def test_user_step_replays_reference(name, steps, envs):
    """AllStepManager(UserTeamBattle) replays the reference's golden
    trajectories, one env at a time, bit-exactly."""
    from tests.cases import load_golden, build_sim
    g = load_golden(name)
    c = g['case']
    S = g['obs0'].shape[-1]
    for e in range(envs):
        sim = build_sim(c, sim_cls=UserTeamBattle)
        sim.len_fix = bool(c.get('len_fix'))
        assert sim._engine_program is None
        m = AllStepManager(sim)
        ids = list(m.agents)
        np.random.seed(c['seeds'][e])
        obs = m.reset()
        np.testing.assert_array_equal(_obs_array(obs, ids, S), g['obs0'][e], err_msg='reset obs')
        for t in range(steps):
            acts = {aid: {'move': g['actions'][t, e, i, :2].astype(int),
                          'attack': int(g['actions'][t, e, i, 2])}
                    for i, aid in enumerate(ids) if aid not in m.done_agents}
            where = f'{name} env {e} step {t}'
            if 'err' in g and g['err'][t, e]:
                # the reference's step raised ValueError (team_battle_example.py:41)
                with pytest.raises(ValueError):
                    m.step(acts)
                st = np.random.get_state()
                assert st[2] == g['mt_pos'][t, e], where
                assert zlib.crc32(np.ascontiguousarray(st[1], dtype=np.uint32).tobytes()) == \
                    int(g['mt_crc'][t, e]), where
                obs = m.reset()
                np.testing.assert_array_equal(_obs_array(obs, ids, S), g['reset_obs'][t, e],
                                              err_msg=where + ' reset')
                continue
            obs, rew, done, _ = m.step(acts)
            np.testing.assert_array_equal(_obs_array(obs, ids, S), g['obs'][t, e], err_msg=where)
            for i, aid in enumerate(ids):
                if aid in rew:
                    assert np.float64(rew[aid]).view(np.uint64) == \
                        np.float64(g['reward'][t, e, i]).view(np.uint64), where
                    assert int(bool(done[aid])) == g['done'][t, e, i], where
                a = m.agents[aid]
                assert tuple(a.position) == tuple(g['pos'][t, e, i]), where
                assert getattr(a, 'health', 0.0) == g['health'][t, e, i], where
                assert int(a.active) == g['active'][t, e, i], where
                if 'ammo' in g and isinstance(a, AmmoAgent):
                    assert a.ammo == g['ammo'][t, e, i], where
            assert int(bool(done['__all__'])) == g['all_done'][t, e], where
            st = np.random.get_state()
            assert st[2] == g['mt_pos'][t, e], where
            assert zlib.crc32(np.ascontiguousarray(st[1], dtype=np.uint32).tobytes()) == \
                int(g['mt_crc'][t, e]), where
            if g['reset_mask'][t, e]:
                obs = m.reset()
                np.testing.assert_array_equal(_obs_array(obs, ids, S), g['reset_obs'][t, e],
                                              err_msg=where + ' reset')


# ------------------------------ ReachTheTarget, BASELINE config 4, user step
def _user_rtt_class():
    """Test-side user code: the reference's ReachTheTarget example
    (examples/sim/reach_the_target.py:84-158) written against this
    repository's components, dones as plain reads of the agents."""
    from abmarl_amd.sim.agent_based_simulation import Agent
    from abmarl_amd.sim.gridworld.base import GridWorldSimulation
    from abmarl_amd.examples.reach_the_target import RunningAgent, TargetAgent

    class UserReachTheTarget(GridWorldSimulation):
        def __init__(self, **kw):
            super().__init__(**kw)
            self.target = self.agents['target']
            self.position_state = PositionState(**kw)
            self.health_state = HealthState(**kw)
            self.move_actor = MoveActor(**kw)
            self.attack_actor = SelectiveAttackActor(**kw)
            self.observer = PositionCenteredEncodingObserver(**kw)
            self.finalize()

        def reset(self, **kw):
            self.health_state.reset(**kw)
            self.position_state.reset(**kw)
            self.rewards = {a.id: 0 for a in self.agents.values() if isinstance(a, Agent)}

        def _on_target(self, agent):
            return agent is not self.target and np.array_equal(agent.position, self.target.position)

        def _left(self):
            return sum(1 for a in self.agents.values() if a.active and isinstance(a, Agent))

        def step(self, action_dict, **kw):
            for aid, action in action_dict.items():
                agent = self.agents[aid]
                if not agent.active:
                    continue
                status, hit = self.attack_actor.process_action(agent, action, **kw)
                if status and not hit:
                    self.rewards[aid] -= 0.1
                for other in hit:
                    if not other.active:
                        self.rewards[other.id] -= 1
                        self.rewards[aid] += 1
            for aid, action in action_dict.items():
                agent = self.agents[aid]
                if not isinstance(agent, MovingAgent):
                    continue
                if agent.active and not self.move_actor.process_action(agent, action, **kw):
                    self.rewards[aid] -= 0.1
                if self._on_target(agent):
                    self.rewards[aid] += 1
                    self.grid.remove(agent, agent.position)
                    agent.active = False
            for aid in action_dict:
                if isinstance(self.agents[aid], RunningAgent):
                    self.rewards[aid] -= 0.01

        def get_obs(self, aid, **kw):
            return dict(self.observer.get_obs(self.agents[aid], **kw))

        def get_reward(self, aid, **kw):
            r, self.rewards[aid] = self.rewards[aid], 0
            return r

        def get_done(self, aid, **kw):
            agent = self.agents[aid]
            if isinstance(agent, RunningAgent):
                return not agent.active or self._on_target(agent)
            if isinstance(agent, TargetAgent):
                return self._left() <= 1

        def get_all_done(self, **kw):
            return self._left() <= 1

        def get_info(self, aid, **kw):
            return {}

    return UserReachTheTarget


@gpu
def test_user_rtt_config4_replays_reference(component_kernel):
    """BASELINE config 4's grid (64x64, 128 barriers + 127 runners + the
    target = 256 entities: the workgroup-per-env component kernel) driven
    by a user-written step() through MultiAgentWrapper(AllStepManager), one
    component call at a time, against the reference's own trajectory
    (tests/golden/rtt_64.npz): observations, reward bits, dones, positions,
    health and the numpy stream after every step."""
    if component_kernel != 'wave':
        pytest.skip('256 entities always run on the workgroup kernel')
    from abmarl_amd.external import MultiAgentWrapper
    from abmarl_amd.sim.agent_based_simulation import Agent
    from tests.cases import load_golden, build_rtt
    from tests.test_dict_api import _check_obs, _action
    g = load_golden('rtt_64')
    c = g['case']
    steps = 12
    for e in range(2):
        sim = build_rtt(c, sim_cls=_user_rtt_class())
        ids = list(sim.agents)
        index = {k: i for i, k in enumerate(ids)}
        agents0 = np.array([isinstance(a, Agent) for a in sim.agents.values()])
        env = MultiAgentWrapper(AllStepManager(sim))
        np.random.seed(c['seeds'][e])
        obs = env.reset()
        from abmarl_amd.sim.gridworld.component_runtime import ComponentRuntime
        rt = ComponentRuntime.of(sim.observer)
        assert rt.eng.wg and len(rt.lane_ids) == 256
        _check_obs(obs, g['obs0'][e], agents0, index)
        for t in range(steps):
            done_agents = env.sim.done_agents
            adict = {k: _action(sim.agents[k], g['actions'][t, e, i])
                     for i, k in enumerate(ids) if k not in done_agents}
            assert not g['err'][t, e]
            o, r, d, _ = env.step(adict)
            _check_obs(o, g['obs'][t, e], g['returned'][t, e], index)
            for k, v in r.items():
                i = index[k]
                assert np.float64(v).view(np.uint64) == g['reward'][t, e, i].view(np.uint64), (t, k)
                assert bool(d[k]) == bool(g['done'][t, e, i]), (t, k)
            assert bool(d['__all__']) == bool(g['all_done'][t, e])
            st = np.random.get_state()
            assert st[2] == g['mt_pos'][t, e]
            assert zlib.crc32(np.ascontiguousarray(st[1], np.uint32).tobytes()) == g['mt_crc'][t, e]
            for i, agent in enumerate(sim.agents.values()):
                np.testing.assert_array_equal(agent.position, g['pos'][t, e, i])
                assert getattr(agent, 'health', 0.0) == g['health'][t, e, i]
            assert not g['reset_mask'][t, e]


# -------------------------------------------------------------------- CPU
def test_attack_mapping_validation():
    """test_actor.py:503-528: malformed attack mappings are rejected at construction."""
    grid = Grid(5, 6)
    agents = _attack_agents(dict(attack_strength=1, attack_accuracy=1))
    for bad in ([1, 2, 3], {'1': {3}, 2.0: {6}}, {1: 3, 2: [6]}, {1: {'2', 3}, 2: {2, 3}}):
        with pytest.raises(AssertionError):
            BinaryAttackActor(agents=agents, grid=grid, attack_mapping=bad)


def test_component_spaces():
    """Action / observation spaces the components assign (test_actor.py:43-46,
    test_observer.py:216-224)."""
    from abmarl_amd.spaces import Box, Discrete
    grid = Grid(5, 5)
    agents = _observer_agents(False)
    PositionCenteredEncodingObserver(agents=agents, grid=grid)
    assert agents['agent0'].observation_space[KEY] == Box(-2, 6, (5, 5), int)
    assert agents['agent1'].observation_space[KEY] == Box(-2, 6, (3, 3), int)
    assert agents['agent2'].observation_space[KEY] == Box(-2, 6, (9, 9), int)
    agents = _attack_agents(dict(attack_strength=1, attack_accuracy=1, simultaneous_attacks=3))
    BinaryAttackActor(attack_mapping={1: {1}}, grid=Grid(5, 6), agents=agents)
    assert agents['agent1'].action_space['attack'] == Discrete(4)


def test_runtime_needs_the_engine():
    """The component path has no host fallback: without a GPU it fails."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    grid = Grid(3, 3)
    agents = {'agent0': GridWorldAgent(id='agent0', encoding=1)}
    with pytest.raises(Exception):
        PositionState(grid=grid, agents=agents).reset()
