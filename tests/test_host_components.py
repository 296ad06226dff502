"""The five registry components that run on the host (host_components.py):
EncodingBasedAttackActor, RestrictedSelectiveAttackActor,
StackedPositionCenteredEncodingObserver, AbsolutePositionObserver,
AmmoObserver.

The scenarios and known answers are the reference's own unit tests
(tests/sim/gridworld/test_actor.py:1175-1709, test_observer.py:15-40,
342-640, 906-1060), restated.  Their grids hold only agents with initial
positions, so the placement needs no draw: the CPU tests reset the Grid and
place the agents on the host (PositionState.reset's first pass, state.py:
103-112) and draw missing health with np.random.uniform in agent order
(HealthState.reset, state.py:629-641); the GPU tests run the built-in
PositionState / HealthState as device operations instead and then the host
components on what they left (the component runtime's mirror and stream
hand-over).
"""
import numpy as np
import pytest

from abmarl_amd.spaces import Box, Dict, Discrete, MultiDiscrete
from abmarl_amd.sim.agent_based_simulation import ObservingAgent
from abmarl_amd.sim.gridworld.grid import Grid
from abmarl_amd.sim.gridworld.agent import (
    GridWorldAgent, GridObservingAgent, AttackingAgent, HealthAgent, AmmoAgent, AmmoObservingAgent)
from abmarl_amd.sim.gridworld.components import (
    ActorBaseComponent, ObserverBaseComponent, PositionState, HealthState, AmmoState)
from abmarl_amd.sim.gridworld.host_components import (
    EncodingBasedAttackActor, RestrictedSelectiveAttackActor, StackedPositionCenteredEncodingObserver,
    AbsolutePositionObserver, AmmoObserver)


class Gunner(AttackingAgent, AmmoAgent):
    pass


@pytest.fixture(params=['host', pytest.param('device', marks=pytest.mark.gpu)])
def resetter(request):
    """reset(grid, agents): the initial-position placement and the health
    reset, on the host or as the built-in device operations."""
    def host(grid, agents):
        grid.reset()
        for a in agents.values():
            if a.initial_position is not None:
                assert grid.place(a, a.initial_position)
        for a in agents.values():
            if isinstance(a, HealthAgent):
                a.health = a.initial_health if a.initial_health is not None else np.random.uniform(0, 1)

    def device(grid, agents):
        PositionState(grid=grid, agents=agents).reset()
        if any(isinstance(a, HealthAgent) for a in agents.values()):
            HealthState(grid=grid, agents=agents).reset()
    return host if request.param == 'host' else device


def _corner_agents(attacker, fifth=True, health=None):
    """The 2x2 grids of the reference's attack tests: encoding-1 agent0 at
    (0, 0), encoding-2 agent1 / agent2 at (0, 1) / (1, 0), the encoding-3
    attacker at (1, 1) and (optionally) encoding-1 agent4 on `fifth`'s cell."""
    kw = {} if health is None else {'initial_health': health}
    agents = {
        'agent0': HealthAgent(id='agent0', initial_position=np.array([0, 0]), encoding=1, **kw),
        'agent1': HealthAgent(id='agent1', initial_position=np.array([0, 1]), encoding=2, **kw),
        'agent2': HealthAgent(id='agent2', initial_position=np.array([1, 0]), encoding=2, **kw),
        'agent3': attacker,
    }
    if fifth:
        agents['agent4'] = HealthAgent(id='agent4', initial_position=np.array(fifth), encoding=1, **kw)
    return agents


def _attacker(cls=AttackingAgent, **kw):
    return cls(id='agent3', initial_position=np.array([1, 1]), encoding=3, attack_range=1,
               attack_accuracy=1, **kw)


def _check(result, status, encs, active=None, same=False, distinct=False):
    st, hit = result
    assert bool(st) == status
    assert type(hit) is list
    assert [a.encoding for a in hit] == encs
    if active is not None:
        assert [a.active for a in hit] == active
    if same:
        assert hit[0] is hit[1]
    if distinct:
        assert hit[0].id != hit[1].id


# ---------------------------------------------------- EncodingBasedAttackActor
def test_encoding_based(resetter):
    agents = _corner_agents(_attacker(attack_strength=0), fifth=[1, 1])
    grid = Grid(2, 2, overlapping={1: {3}, 3: {1}})
    actor = EncodingBasedAttackActor(attack_mapping={3: {1, 2}}, grid=grid, agents=agents)
    assert isinstance(actor, ActorBaseComponent)
    assert actor.key == 'attack' and actor.supported_agent_type == AttackingAgent
    assert agents['agent3'].action_space['attack'] == Dict({1: Discrete(2), 2: Discrete(2)})
    agents['agent3'].finalize()
    assert agents['agent3'].null_action == {'attack': {1: 0, 2: 0}}
    resetter(grid, agents)
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go({1: 0, 2: 1}), True, [2], [True])          # too weak to kill
    agents['agent3'].attack_strength = 1
    _check(go({1: 1, 2: 0}), True, [1], [False])
    _check(go({1: 1, 2: 1}), True, [1, 2], [False, False])
    _check(go({1: 1, 2: 1}), True, [2], [False])
    _check(go({1: 1, 2: 1}), True, [])


def test_encoding_based_ammo(resetter):
    agents = _corner_agents(_attacker(Gunner, attack_strength=0, initial_ammo=4), fifth=[1, 1])
    grid = Grid(2, 2, overlapping={1: {3}, 3: {1}})
    ammo = AmmoState(grid=grid, agents=agents)
    actor = EncodingBasedAttackActor(attack_mapping={3: {1, 2}}, grid=grid, agents=agents)
    resetter(grid, agents)
    ammo.reset()
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go({1: 0, 2: 1}), True, [2], [True])
    assert agents['agent3'].ammo == 3
    agents['agent3'].attack_strength = 1
    _check(go({1: 1, 2: 0}), True, [1], [False])
    assert agents['agent3'].ammo == 2
    _check(go({1: 1, 2: 1}), True, [1, 2], [False, False])
    assert agents['agent3'].ammo == 0
    _check(go({1: 1, 2: 1}), True, [])
    assert agents['agent3'].ammo == 0


def test_encoding_based_simultaneous(resetter):
    agents = _corner_agents(_attacker(attack_strength=0, simultaneous_attacks=2), fifth=[1, 1])
    grid = Grid(2, 2, overlapping={1: {3}, 3: {1}})
    actor = EncodingBasedAttackActor(attack_mapping={3: {1, 2}}, grid=grid, agents=agents)
    assert agents['agent3'].action_space['attack'] == Dict({1: Discrete(3), 2: Discrete(3)})
    resetter(grid, agents)
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go({1: 0, 2: 0}), False, [])
    for att, encs in [({1: 1, 2: 0}, [1]), ({1: 0, 2: 1}, [2]), ({1: 1, 2: 1}, [1, 2]),
                      ({1: 2, 2: 1}, [1, 1, 2]), ({1: 1, 2: 2}, [1, 2, 2]), ({1: 2, 2: 2}, [1, 1, 2, 2])]:
        _check(go(att), True, encs)
    agents['agent3'].attack_strength = 1
    _check(go({1: 2, 2: 0}), True, [1, 1], [False, False])
    _check(go({1: 2, 2: 2}), True, [2, 2], [False, False])
    _check(go({1: 1, 2: 1}), True, [])


def test_encoding_based_stacked(resetter):
    agents = _corner_agents(_attacker(attack_strength=1, simultaneous_attacks=2), fifth=[1, 1])
    grid = Grid(2, 2, overlapping={1: {3}, 3: {1}})
    actor = EncodingBasedAttackActor(attack_mapping={3: {1, 2}}, stacked_attacks=True, grid=grid,
                                     agents=agents)
    resetter(grid, agents)
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go({1: 1, 2: 1}), True, [1, 2], [False, False])
    _check(go({1: 2, 2: 0}), True, [1, 1], [False, False], same=True)
    _check(go({1: 2, 2: 2}), True, [2, 2], [False, False], same=True)


# --------------------------------------------- RestrictedSelectiveAttackActor
def test_restricted_selective(resetter):
    agents = _corner_agents(_attacker(attack_strength=0, simultaneous_attacks=2), fifth=[0, 0])
    grid = Grid(2, 2, overlapping={1: {1}})
    actor = RestrictedSelectiveAttackActor(attack_mapping={3: {1, 2}}, grid=grid, agents=agents)
    assert isinstance(actor, ActorBaseComponent) and actor.key == 'attack'
    assert agents['agent3'].action_space['attack'] == MultiDiscrete([10, 10])
    agents['agent3'].finalize()
    np.testing.assert_array_equal(agents['agent3'].null_action['attack'], np.zeros((2,), dtype=int))
    resetter(grid, agents)
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go([0, 0]), False, [])
    # code 1: window cell (0, 0) = grid (0, 0), two encoding-1 agents, two distinct picks
    _check(go([1, 1]), True, [1, 1], [True, True], distinct=True)
    # code 2: window cell (1, 0) = grid (1, 0): agent2 only, not hit twice
    _check(go([2, 2]), True, [2], [True])
    # code 4: window cell (0, 1) = grid (0, 1)
    _check(go([1, 4]), True, [1, 2], [True, True])


def test_restricted_selective_stacked(resetter):
    agents = _corner_agents(_attacker(attack_strength=1, simultaneous_attacks=2), fifth=False, health=1)
    grid = Grid(2, 2, overlapping={1: {1}})
    actor = RestrictedSelectiveAttackActor(attack_mapping={3: {1, 2}}, stacked_attacks=True, grid=grid,
                                           agents=agents)
    resetter(grid, agents)
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go([0, 0]), False, [])
    _check(go([1, 1]), True, [1, 1], [False, False], same=True)
    _check(go([2, 2]), True, [2, 2], [False, False], same=True)
    _check(go([4, 4]), True, [2, 2], [False, False], same=True)


def test_restricted_selective_ammo(resetter):
    agents = _corner_agents(_attacker(Gunner, attack_strength=1, simultaneous_attacks=2, initial_ammo=1),
                            fifth=False, health=1)
    grid = Grid(2, 2, overlapping={1: {1}})
    ammo = AmmoState(grid=grid, agents=agents)
    actor = RestrictedSelectiveAttackActor(attack_mapping={3: {1, 2}}, stacked_attacks=True, grid=grid,
                                           agents=agents)
    resetter(grid, agents)
    ammo.reset()
    go = lambda a: actor.process_action(agents['agent3'], {'attack': a})
    _check(go([0, 0]), False, [])
    _check(go([1, 1]), True, [1], [False])               # one round of ammo
    assert agents['agent3'].ammo == 0
    _check(go([2, 2]), True, [])
    assert agents['agent3'].ammo == 0


def test_draws_follow_the_reference_order():
    """The accuracy draws (one per candidate passing the id / active /
    mapping tests, in window order) and the subset draw come from the global
    numpy stream in the reference's order: a half-accuracy attacker's
    outcome equals the same sequence of np.random calls made by hand."""
    def run():
        agents = _corner_agents(_attacker(attack_strength=0, simultaneous_attacks=2), fifth=[1, 1],
                                health=1)
        agents['agent3'].attack_accuracy = 0.5
        grid = Grid(2, 2, overlapping={1: {3}, 3: {1}})
        actor = EncodingBasedAttackActor(attack_mapping={3: {1, 2}}, grid=grid, agents=agents)
        grid.reset()
        for a in agents.values():
            grid.place(a, a.initial_position)
            if isinstance(a, HealthAgent):
                a.health = 1
        return agents, actor
    np.random.seed(7)
    agents, actor = run()
    got = [[a.id for a in actor.process_action(agents['agent3'], {'attack': {1: 1, 2: 2}})[1]]
           for _ in range(6)]
    np.random.seed(7)
    want = []
    # window of agent3 at (1, 1), range 1 on a 2x2 grid: cells (0,0) (0,1) (1,0) (1,1)
    order = ['agent0', 'agent1', 'agent2', 'agent3', 'agent4']
    enc = {'agent0': 1, 'agent1': 2, 'agent2': 2, 'agent4': 1}
    for _ in range(6):
        pools = {1: [], 2: []}
        for aid in order:
            if aid == 'agent3':
                continue
            if not np.random.uniform() > 0.5:
                pools[enc[aid]].append(aid)
        out = []
        for e, n in ((1, 1), (2, 2)):
            if pools[e]:
                out.extend(pools[e] if n > len(pools[e]) else list(np.random.choice(pools[e], size=n,
                                                                                    replace=False)))
        want.append(out)
    assert got == want


# ------------------------------------------------------------------ observers
def test_ammo_observer():
    grid = Grid(3, 3)
    agents = {
        'agent0': AmmoAgent(id='agent0', encoding=1, initial_ammo=10),
        'agent1': AmmoObservingAgent(id='agent1', encoding=1, initial_ammo=-3),
        'agent2': AmmoObservingAgent(id='agent2', encoding=1, initial_ammo=14),
        'agent3': AmmoObservingAgent(id='agent3', encoding=1, initial_ammo=12),
    }
    state = AmmoState(grid=grid, agents=agents)
    observer = AmmoObserver(grid=grid, agents=agents)
    assert isinstance(observer, ObserverBaseComponent)
    state.reset()
    for k in ('agent1', 'agent2', 'agent3'):
        assert observer.get_obs(agents[k])['ammo'] == agents[k].ammo
    assert agents['agent1'].ammo == 0                     # initial -3 clamps to 0
    agents['agent0'].ammo -= 16
    agents['agent1'].ammo += 7
    agents['agent2'].ammo -= 15
    for k in ('agent1', 'agent2', 'agent3'):
        assert observer.get_obs(agents[k])['ammo'] == agents[k].ammo
    assert [agents[k].ammo for k in ('agent1', 'agent2', 'agent3')] == [7, 0, 12]
    assert not observer.get_obs(agents['agent0'])
    assert isinstance(Gunner(id='g', encoding=1, attack_range=1, attack_strength=1, attack_accuracy=1,
                             initial_ammo=1), AmmoAgent)
    assert not isinstance(agents['agent0'], AmmoObservingAgent)
    assert agents['agent2'].observation_space['ammo'] == Box(0, 14, (1,), int)


def test_absolute_position_observer(resetter):
    class Locator(ObservingAgent, GridWorldAgent):
        pass
    grid = Grid(6, 7, overlapping={1: {5}, 4: {6}, 5: {1}, 6: {4}})
    cells = [(0, 0), (5, 0), (0, 6), (5, 6), (0, 0), (5, 6)]
    agents = {f'agent{i}': Locator(id=f'agent{i}', encoding=i + 1, initial_position=np.array(rc))
              for i, rc in enumerate(cells)}
    observer = AbsolutePositionObserver(agents=agents, grid=grid)
    assert observer.key == 'position' and observer.supported_agent_type == ObservingAgent
    assert isinstance(observer, ObserverBaseComponent)
    for a in agents.values():
        a.finalize()
        assert a.observation_space['position'] == Box(np.array([0, 0]), np.array([5, 6]), dtype=int)
        np.testing.assert_array_equal(a.null_observation['position'], np.array([0, 0]))
    resetter(grid, agents)
    for i, rc in enumerate(cells):
        np.testing.assert_array_equal(observer.get_obs(agents[f'agent{i}'])['position'], np.array(rc))


@pytest.mark.gpu
def test_absolute_position_beside_the_device_observer():
    """test_observer.py:986-1060: the host observer next to the built-in
    PositionCenteredEncodingObserver (a device operation) on one grid."""
    from abmarl_amd.sim.gridworld.components import PositionCenteredEncodingObserver
    grid = Grid(6, 7, overlapping={1: {5}, 4: {6}, 5: {1}, 6: {4}})
    agents = {
        'agent0': GridObservingAgent(id='agent0', encoding=1, initial_position=np.array([2, 2]), view_range=2),
        'agent1': GridObservingAgent(id='agent1', encoding=2, initial_position=np.array([3, 4]), view_range=2),
        'agent2': GridWorldAgent(id='agent2', encoding=3, initial_position=np.array([0, 0])),
        'agent3': GridWorldAgent(id='agent3', encoding=4, initial_position=np.array([5, 6])),
        'agent4': GridWorldAgent(id='agent4', encoding=5, initial_position=np.array([4, 3])),
    }
    position_state = PositionState(grid=grid, agents=agents)
    grid_observer = PositionCenteredEncodingObserver(grid=grid, agents=agents)
    position_observer = AbsolutePositionObserver(grid=grid, agents=agents)
    for aid in ('agent0', 'agent1'):
        a = agents[aid]
        a.finalize()
        assert a.observation_space['position'] == Box(np.array([0, 0]), np.array([5, 6]), dtype=int)
        assert a.observation_space['position_centered_encoding'] == Box(-2, 5, (5, 5), int)
    position_state.reset()
    np.testing.assert_array_equal(position_observer.get_obs(agents['agent0'])['position'], [2, 2])
    np.testing.assert_array_equal(
        grid_observer.get_obs(agents['agent0'])['position_centered_encoding'],
        [[3, 0, 0, 0, 0], [0, 0, 0, 0, 0], [0, 0, 1, 0, 0], [0, 0, 0, 0, 2], [0, 0, 0, 5, 0]])
    np.testing.assert_array_equal(position_observer.get_obs(agents['agent1'])['position'], [3, 4])
    np.testing.assert_array_equal(
        grid_observer.get_obs(agents['agent1'])['position_centered_encoding'],
        [[0, 0, 0, 0, 0], [1, 0, 0, 0, 0], [0, 0, 2, 0, 0], [0, 5, 0, 0, 0], [0, 0, 0, 0, 4]])


def _stacked_agents(blocking):
    """test_observer.py:342-375 / 609-640: 9 agents on a 5x5 grid, encodings
    1-6; agents 3, 8, 4, 5 block in the blocking variant."""
    from abmarl_amd.sim.gridworld.agent import MovingAgent

    class Roamer(GridObservingAgent, MovingAgent):
        pass
    b = dict(blocking=True) if blocking else {}
    P = lambda r, c: np.array([r, c])
    return {
        'agent0': GridObservingAgent(id='agent0', encoding=1, view_range=2, initial_position=P(2, 2)),
        'agent1': GridObservingAgent(id='agent1', encoding=2, view_range=1, initial_position=P(0, 0)),
        'agent2': GridObservingAgent(id='agent2', encoding=3, view_range=4, initial_position=P(4, 4)),
        'agent6': Roamer(id='agent6', encoding=2, view_range=1, initial_position=P(4, 4), move_range=1),
        'agent7': Roamer(id='agent7', encoding=3, view_range=4, initial_position=P(0, 0), move_range=1),
        'agent3': GridWorldAgent(id='agent3', encoding=5, initial_position=P(3, 3), **b),
        'agent8': MovingAgent(id='agent8', encoding=5, initial_position=P(3, 3), move_range=1, **b),
        'agent4': GridWorldAgent(id='agent4', encoding=4, initial_position=P(1, 1), **b),
        'agent5': GridWorldAgent(id='agent5', encoding=6, initial_position=P(2, 1), **b),
    }


# occupants per grid cell (encoding -> count) of that scenario
_STACKED_CELLS = {(2, 2): {1: 1}, (0, 0): {2: 1, 3: 1}, (4, 4): {2: 1, 3: 1}, (3, 3): {5: 2},
                  (1, 1): {4: 1}, (2, 1): {6: 1}}


def _stacked_expected(center, view, hidden=()):
    """The (2v+1, 2v+1, 6) observation from the scenario's occupants: -1 off
    the grid, -2 on the hidden window cells (the reference's known masks),
    else the per-encoding counts."""
    side = 2 * view + 1
    out = np.zeros((side, side, 6), dtype=int)
    for wr in range(side):
        for wc in range(side):
            r, c = center[0] - view + wr, center[1] - view + wc
            if (wr, wc) in hidden:
                out[wr, wc] = -2
            elif not (0 <= r < 5 and 0 <= c < 5):
                out[wr, wc] = -1
            else:
                for e, n in _STACKED_CELLS.get((r, c), {}).items():
                    out[wr, wc, e - 1] = n
    return out


def _hidden(rows):
    """window cells marked '#' in a picture of the mask"""
    return {(r, c) for r, row in enumerate(rows) for c, ch in enumerate(row) if ch == '#'}


def test_stacked_observer(resetter):
    agents = _stacked_agents(blocking=False)
    grid = Grid(5, 5, overlapping={2: {3}, 3: {2}, 5: {5}})
    observer = StackedPositionCenteredEncodingObserver(agents=agents, grid=grid)
    key = 'stacked_position_centered_encoding'
    assert observer.key == key and observer.supported_agent_type == GridObservingAgent
    assert isinstance(observer, ObserverBaseComponent)
    assert observer.number_of_encodings == 6
    for aid, side in (('agent0', 5), ('agent1', 3), ('agent2', 9)):
        assert agents[aid].observation_space[key] == Box(-2, 9, (side, side, 6), int)
        agents[aid].finalize()
        assert agents[aid].null_observation.keys() == {key}
        np.testing.assert_array_equal(agents[aid].null_observation[key], -2 * np.ones((side, side, 6)))
    resetter(grid, agents)
    for aid, center, view in (('agent0', (2, 2), 2), ('agent1', (0, 0), 1), ('agent2', (4, 4), 4)):
        np.testing.assert_array_equal(observer.get_obs(agents[aid])[key], _stacked_expected(center, view))
    assert observer.get_obs(agents['agent3']) == {}


def test_stacked_observer_blocking(resetter):
    agents = _stacked_agents(blocking=True)
    grid = Grid(5, 5, overlapping={2: {3}, 3: {2}, 5: {5}})
    observer = StackedPositionCenteredEncodingObserver(agents=agents, grid=grid)
    key = 'stacked_position_centered_encoding'
    resetter(grid, agents)
    # the reference's masks (test_observer.py:648-843), '#' hidden in every layer
    m0 = _hidden(['##...', '#....', '#....', '#...#', '...##'])
    m2 = _hidden(['###..', '###..', '####.', '..#..', '.....'])
    np.testing.assert_array_equal(observer.get_obs(agents['agent0'])[key], _stacked_expected((2, 2), 2, m0))
    np.testing.assert_array_equal(observer.get_obs(agents['agent1'])[key], _stacked_expected((0, 0), 1))
    np.testing.assert_array_equal(observer.get_obs(agents['agent2'])[key], _stacked_expected((4, 4), 4, m2))


def test_registry_names_match_the_reference():
    """registry.py:20-47 of the reference: the same names per kind."""
    from abmarl_amd.sim.gridworld.registry import registry
    assert {k: sorted(v) for k, v in registry.items()} == {
        'actor': ['BinaryAttackActor', 'CrossMoveActor', 'DriftMoveActor', 'EncodingBasedAttackActor',
                  'MoveActor', 'RestrictedSelectiveAttackActor', 'SelectiveAttackActor'],
        'done': ['ActiveDone', 'OneTeamRemainingDone', 'TargetAgentDone', 'TargetDestroyedDone'],
        'observer': ['AbsoluteEncodingObserver', 'AbsolutePositionObserver', 'AmmoObserver',
                     'PositionCenteredEncodingObserver', 'StackedPositionCenteredEncodingObserver'],
        'state': ['AmmoState', 'HealthState', 'MazePlacementState', 'OrientationState', 'PositionState',
                  'TargetBarriersFreePlacementState']}


def test_fused_programs_refuse_host_components():
    from abmarl_amd.examples import TeamBattleSim
    from abmarl_amd.sim.gridworld.compile import UnsupportedConfig
    from tests.cases import Fighter
    agents = {f'a{i}': Fighter(id=f'a{i}', encoding=1 + i % 2, move_range=1, attack_range=1,
                               attack_strength=1, attack_accuracy=1, view_range=2) for i in range(4)}
    sim = TeamBattleSim.build_sim(5, 5, agents=agents, attack_mapping={1: {2}, 2: {1}},
                                  states={'PositionState', 'HealthState'},
                                  observers={'StackedPositionCenteredEncodingObserver'},
                                  dones={'OneTeamRemainingDone'})
    with pytest.raises(UnsupportedConfig):
        sim.compiled()
