"""The component registry accepts user components (registry.py:58-77) and a
simulation mixing them with the built-in ones runs: the user's Python on the
host Grid / agents, the built-in components as device operations.

Evidence:
  * the reference's tests/sim/gridworld/test_registry.py restated (built-ins
    registered, user classes registered by type and name, a non-component
    refused with TypeError);
  * create_grid_and_mask (the host form user components call) against 400
    masks the reference computed (tests/golden/make_masks.py);
  * on the GPU, a simulation built from user components (tests/user_lanterns.py:
    lantern keepers sharing oil in sight of each other, blocking wanderers)
    replays the trajectory the reference's built-ins produced with the same
    user code (tests/golden/make_comms.py): grid windows, oil readings,
    rewards, dones, positions and the numpy stream.
"""
import json
import os
import types
import zlib

import numpy as np
import pytest

from abmarl_amd.sim.gridworld.registry import registry, register
from abmarl_amd.sim.gridworld import components as comp
from tests import user_lanterns

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def our_namespace():
    from abmarl_amd.sim.agent_based_simulation import ObservingAgent, ActingAgent
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent, MovingAgent, GridObservingAgent
    from abmarl_amd.sim.gridworld.base import GridWorldSimulation
    from abmarl_amd.sim.gridworld.components import (
        StateBaseComponent, PositionState, ActorBaseComponent, MoveActor, ObserverBaseComponent,
        PositionCenteredEncodingObserver, DoneBaseComponent)
    from abmarl_amd.sim.gridworld.utils import create_grid_and_mask
    from abmarl_amd.spaces import Box, Discrete, Dict
    return types.SimpleNamespace(**{k: v for k, v in locals().items()})


def test_built_in_registry():
    """test_registry.py:19-40 (the built-ins this repository implements)."""
    for kind, cls in [('actor', comp.MoveActor), ('actor', comp.CrossMoveActor),
                      ('actor', comp.DriftMoveActor), ('actor', comp.BinaryAttackActor),
                      ('actor', comp.SelectiveAttackActor), ('done', comp.ActiveDone),
                      ('done', comp.TargetAgentDone), ('done', comp.TargetDestroyedDone),
                      ('done', comp.OneTeamRemainingDone), ('observer', comp.AbsoluteEncodingObserver),
                      ('observer', comp.PositionCenteredEncodingObserver), ('state', comp.PositionState),
                      ('state', comp.TargetBarriersFreePlacementState), ('state', comp.MazePlacementState),
                      ('state', comp.HealthState), ('state', comp.AmmoState),
                      ('state', comp.OrientationState)]:
        assert cls in registry[kind].values(), cls.__name__


def test_custom_registrations():
    """test_registry.py:43-55: user components register by type and name; an
    agent class is not a component."""
    classes = user_lanterns.lantern_classes(our_namespace())
    for k in user_lanterns.USER_COMPONENTS:
        register(classes[k])
    assert classes['OilStock'] in registry['state'].values()
    assert classes['PourActor'] in registry['actor'].values()
    assert classes['OilGauge'] in registry['observer'].values()
    assert classes['EvenOilDone'] in registry['done'].values()
    assert registry['actor']['PourActor'] is classes['PourActor']
    with pytest.raises(TypeError):
        register(classes['Keeper'])


def test_program_sims_refuse_user_components():
    """A fused engine program compiles the built-in components only: a user
    state in its sets is refused when the program compiles."""
    from abmarl_amd.examples import TeamBattleSim
    from abmarl_amd.sim.gridworld.compile import UnsupportedConfig
    from tests.cases import Fighter
    classes = user_lanterns.lantern_classes(our_namespace())
    register(classes['OilStock'])
    agents = {f'a{i}': Fighter(id=f'a{i}', encoding=1 + i % 2, move_range=1, attack_range=1,
                               attack_strength=1, attack_accuracy=1, view_range=2) for i in range(4)}
    sim = TeamBattleSim.build_sim(5, 5, agents=agents, attack_mapping={1: {2}, 2: {1}},
                                  states={'PositionState', 'HealthState', 'OilStock'},
                                  observers={'PositionCenteredEncodingObserver'},
                                  dones={'OneTeamRemainingDone'})
    with pytest.raises(UnsupportedConfig):
        sim.compiled()


def test_create_grid_and_mask_known_answers():
    """The host create_grid_and_mask (user components' utility) against the
    reference's own masks for 400 random grids with blocking agents."""
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent
    from abmarl_amd.sim.gridworld.grid import Grid
    from abmarl_amd.sim.gridworld.utils import create_grid_and_mask
    z = np.load(os.path.join(GOLDEN, 'masks.npz'))
    for k in range(z['meta'].shape[0]):
        R, C, mr, nb = (int(x) for x in z['meta'][k])
        grid = Grid(R, C)
        grid.reset()
        agents = {}
        for i, x in enumerate(z['cells'][k, :nb + 1]):
            a = GridWorldAgent(id=f'a{i}', encoding=1, blocking=i > 0,
                               initial_position=np.array([int(x) // C, int(x) % C]))
            grid.place(a, (int(x) // C, int(x) % C))
            agents[a.id] = a
        local, mask = create_grid_and_mask(agents['a0'], grid, mr, agents)
        d = 2 * mr + 1
        np.testing.assert_array_equal(mask, z['masks'][k, :d, :d], err_msg=f'case {k}')
        # the local grid: the cells around the observer, None off the grid
        r0, c0 = agents['a0'].position
        for r in range(d):
            for c in range(d):
                gr, gc = r0 - mr + r, c0 - mr + c
                inside = 0 <= gr < R and 0 <= gc < C
                assert (local[r, c] is grid[gr, gc]) if inside else local[r, c] is None


@pytest.mark.gpu
def test_user_components_replay_reference():
    """A simulation of user components (host Python) and built-in components
    (device operations) under AllStepManager replays the reference's
    trajectory of the same user code bit-exactly."""
    from abmarl_amd.managers import AllStepManager
    from abmarl_amd.sim.gridworld.component_runtime import ComponentRuntime
    d = json.load(open(os.path.join(GOLDEN, 'lanterns.json')))
    classes = user_lanterns.lantern_classes(our_namespace())
    for k in user_lanterns.USER_COMPONENTS:
        register(classes[k])
    h = float.fromhex

    def check(sim, obs, rec, where):
        for aid, want in rec['obs'].items():
            got = obs[aid]
            if 'grid' in want:
                np.testing.assert_array_equal(got['position_centered_encoding'], np.array(want['grid']),
                                              err_msg=where)
            if 'oil' in want:
                assert [float(v) for v in got['oil']] == [h(v) for v in want['oil']], where
        assert set(obs) == set(rec['obs']), where
        for aid, p in rec['pos'].items():
            assert list(map(int, sim.agents[aid].position)) == p, where
        for aid, v in rec['oil'].items():
            assert sim.agents[aid].oil == h(v), where
        st = np.random.get_state()
        assert st[2] == rec['mt_pos'], where
        assert zlib.crc32(np.ascontiguousarray(st[1], dtype=np.uint32).tobytes()) == rec['mt_crc'], where

    for env in d['envs']:
        sim = user_lanterns.build(classes)
        m = AllStepManager(sim)
        np.random.seed(env['seed'])
        check(sim, m.reset(), env['reset'], f"seed {env['seed']} reset")
        rt = ComponentRuntime.of(sim.grid_observer)
        assert rt.eng is not None
        for t, rec in enumerate(env['steps']):
            acts = {k: {kk: (np.array(vv) if kk == 'move' else vv) for kk, vv in v.items()}
                    for k, v in rec['actions'].items()}
            o, r, dn, _ = m.step(acts)
            where = f"seed {env['seed']} step {t}"
            check(sim, o, rec, where)
            assert {k: float(v) for k, v in r.items()} == {k: h(v) for k, v in rec['reward'].items()}, where
            assert {k: bool(v) for k, v in dn.items()} == rec['done'], where


def test_overriding_subclass_of_a_built_in_is_refused():
    """A fused program runs the built-in components' device code: a user
    subclass that overrides one of their methods (here PositionState.reset)
    would be ignored silently, so compiling refuses it; a subclass that only
    renames keeps compiling."""
    from abmarl_amd.examples import TeamBattleSim
    from abmarl_amd.sim.gridworld.compile import UnsupportedConfig
    from abmarl_amd.sim.gridworld.components import PositionState
    from tests.cases import Fighter

    class MyPosition(PositionState):
        def reset(self, **kwargs):
            super().reset(**kwargs)

    class SamePosition(PositionState):
        pass

    register(MyPosition)
    register(SamePosition)
    agents = {f'a{i}': Fighter(id=f'a{i}', encoding=1 + i % 2, move_range=1, attack_range=1,
                               attack_strength=1, attack_accuracy=1, view_range=2) for i in range(4)}
    kw = dict(agents=agents, attack_mapping={1: {2}, 2: {1}}, observers={'PositionCenteredEncodingObserver'},
              dones={'OneTeamRemainingDone'})
    sim = TeamBattleSim.build_sim(5, 5, states={'MyPosition', 'HealthState'}, **kw)
    with pytest.raises(UnsupportedConfig, match='overrides reset'):
        sim.compiled()
    TeamBattleSim.build_sim(5, 5, states={'SamePosition', 'HealthState'}, **kw).compiled()

    # the reference's protected hooks count too (state.py:152, actor.py:394)
    class MyPlacement(PositionState):
        def _place_variable_position_agent(self, var_agent_to_place, **kwargs):
            pass

    register(MyPlacement)
    sim = TeamBattleSim.build_sim(5, 5, states={'MyPlacement', 'HealthState'}, **kw)
    with pytest.raises(UnsupportedConfig, match='overrides _place_variable_position_agent'):
        sim.compiled()


def test_attribute_state_twin_is_not_compiled_twice():
    """A simulation that also keeps its own PositionState attribute beside the
    set's compiles (smart.py compiled(): attribute states of a type the sets
    already hold are the same component kind)."""
    from abmarl_amd.examples import TeamBattleSim
    from abmarl_amd.sim.gridworld.components import PositionState
    from tests.cases import Fighter

    class TwinSim(TeamBattleSim):
        def __init__(self, **kwargs):
            super().__init__(**kwargs)
            self.position_twin = PositionState(**kwargs)

    agents = {f'a{i}': Fighter(id=f'a{i}', encoding=1 + i % 2, move_range=1, attack_range=1,
                               attack_strength=1, attack_accuracy=1, view_range=2) for i in range(4)}
    TwinSim.build_sim(5, 5, agents=agents, attack_mapping={1: {2}, 2: {1}},
                      states={'PositionState', 'HealthState'}, observers={'PositionCenteredEncodingObserver'},
                      dones={'OneTeamRemainingDone'}).compiled()
