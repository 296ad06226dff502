"""GridWorldSimulation builders (base.py:38-198), replaying the reference's
tests/sim/gridworld/test_base.py.

The builders are host-side configuration: every assertion and the agents
dict they produce are checked on the CPU.  The reference's tests then reset
the simulation and read the grid; that reset is a PositionState component
call (a device operation), so those parts are GPU tests.
"""
import numpy as np
import pytest

from abmarl_amd.sim.gridworld.agent import GridWorldAgent
from abmarl_amd.sim.gridworld.base import GridWorldSimulation
from abmarl_amd.sim.gridworld.components import PositionState
from abmarl_amd.sim.gridworld.grid import Grid

gpu = pytest.mark.gpu


class MultiAgentGridSim(GridWorldSimulation):
    """Test-side user code shaped like the reference's examples/sim/
    multi_agent_grid_sim.py: a PositionState and nothing else."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.position_state = PositionState(**kwargs)
        self.finalize()

    def reset(self, **kwargs):
        self.position_state.reset()

    def step(self, action_dict, **kwargs):
        pass

    def get_obs(self, agent_id, **kwargs):
        return {}

    def get_reward(self, agent_id, **kwargs):
        return 0

    def get_done(self, agent_id, **kwargs):
        return False

    def get_all_done(self, **kwargs):
        return False

    def get_info(self, agent_id, **kwargs):
        return {}


def _grid_of_four():
    grid = Grid(2, 2)
    grid.reset()
    agents = {f'agent{i}': GridWorldAgent(id=f'agent{i}', encoding=1, initial_position=np.array(p))
              for i, p in enumerate([(0, 0), (0, 1), (1, 0), (1, 1)])}
    for a in agents.values():
        grid.place(a, tuple(a.initial_position))
    return grid, agents


def test_build_from_grid():
    """test_base.py:46-100 (the builder's part)."""
    grid, agents = _grid_of_four()
    sim = MultiAgentGridSim.build_sim_from_grid(grid)
    assert sim.grid.rows == 2 and sim.grid.cols == 2
    assert sim.grid is not grid
    np.testing.assert_array_equal(sim.grid._internal, np.empty((2, 2), dtype=object))
    assert sim.agents == agents
    for aid, p in zip(agents, [(0, 0), (0, 1), (1, 0), (1, 1)]):
        np.testing.assert_array_equal(sim.agents[aid].initial_position, np.array(p))
    with pytest.raises(AssertionError):
        MultiAgentGridSim.build_sim_from_grid(grid._internal)       # not a Grid
    with pytest.raises(AssertionError):
        # the agents' initial positions must match their cells
        agents['agent1'].initial_position = np.array([1, 0])
        agents['agent2'].initial_position = np.array([0, 1])
        MultiAgentGridSim.build_sim_from_grid(grid)


def _extra_setup():
    grid = Grid(2, 2)
    grid.reset()
    agents = {f'agent{i}': GridWorldAgent(id=f'agent{i}', encoding=1, initial_position=np.array(p))
              for i, p in enumerate([(0, 0), (0, 1), (1, 0)])}
    for a in agents.values():
        grid.place(a, tuple(a.initial_position))
    extra = {
        'agent0': GridWorldAgent(id='agent0', encoding=2, initial_position=np.array([0, 1])),
        'agent3': GridWorldAgent(id='agent3', encoding=3, initial_position=np.array([0, 1])),
        'agent4': GridWorldAgent(id='agent4', encoding=4, initial_position=np.array([1, 0])),
        'agent5': GridWorldAgent(id='agent5', encoding=5),
    }
    return grid, agents, extra


def test_build_from_grid_with_extra_agents():
    """test_base.py:103-185 (the builder's part): an agent in the grid wins
    over an extra agent of the same id; the extra dict is updated in place."""
    grid, agents, extra = _extra_setup()
    extra0, extra3, extra4, extra5 = (extra[k] for k in ('agent0', 'agent3', 'agent4', 'agent5'))
    sim = MultiAgentGridSim.build_sim_from_grid(grid, extra_agents=extra,
                                                overlapping={1: {3, 4}, 3: {1}, 4: {1}})
    assert sim.agents == {'agent0': agents['agent0'], 'agent1': agents['agent1'],
                          'agent2': agents['agent2'], 'agent3': extra3, 'agent4': extra4,
                          'agent5': extra5}
    assert sim.agents['agent0'] is not extra0
    assert list(sim.agents) == ['agent0', 'agent3', 'agent4', 'agent5', 'agent1', 'agent2']
    for aid, p in [('agent0', (0, 0)), ('agent1', (0, 1)), ('agent2', (1, 0)), ('agent3', (0, 1)),
                   ('agent4', (1, 0))]:
        np.testing.assert_array_equal(sim.agents[aid].initial_position, np.array(p))
    assert sim.agents['agent5'].initial_position is None
    with pytest.raises(AssertionError):
        MultiAgentGridSim.build_sim_from_grid(grid, extra_agents=[])
    with pytest.raises(AssertionError):
        MultiAgentGridSim.build_sim_from_grid(grid, extra_agents={0: 1})


def test_build_sim_argument_checks():
    """test_base.py:11-43: rows / cols must be positive integers."""
    for rows, cols in [(3.0, 4), (0, 4), (3, -4), (3, '4')]:
        with pytest.raises(AssertionError):
            MultiAgentGridSim.build_sim(rows, cols)


@gpu
def test_build_and_reset():
    """test_base.py:11-30: the reset places the agent at its initial position."""
    agent = GridWorldAgent(id='agent0', encoding=1, initial_position=np.array([0, 0]))
    sim = MultiAgentGridSim.build_sim(3, 4, agents={'agent0': agent})
    np.testing.assert_array_equal(sim.grid._internal, np.empty((3, 4), dtype=object))
    sim.reset()
    want = [[{'agent0': agent}, {}, {}, {}], [{}, {}, {}, {}], [{}, {}, {}, {}]]
    for r in range(3):
        for c in range(4):
            assert sim.grid[r, c] == want[r][c]


@gpu
def test_build_from_grid_reset():
    """test_base.py:46-100: after reset every agent is alone in its cell."""
    grid, agents = _grid_of_four()
    sim = MultiAgentGridSim.build_sim_from_grid(grid)
    sim.reset()
    for aid, p in zip(agents, [(0, 0), (0, 1), (1, 0), (1, 1)]):
        assert next(iter(sim.grid[p].values())) is agents[aid]


@gpu
def test_build_from_grid_with_extra_agents_reset():
    """test_base.py:103-185: the overlapping extras share cells, agent5 takes
    the one empty cell, and without the overlap the reset raises."""
    grid, agents, extra = _extra_setup()
    sim = MultiAgentGridSim.build_sim_from_grid(grid, extra_agents=extra,
                                                overlapping={1: {3, 4}, 3: {1}, 4: {1}})
    sim.reset()
    assert next(iter(sim.grid[0, 0].values())) is agents['agent0']
    assert agents['agent1'] in sim.grid[0, 1].values()
    assert agents['agent2'] in sim.grid[1, 0].values()
    assert extra['agent3'] in sim.grid[0, 1].values()
    assert extra['agent4'] in sim.grid[1, 0].values()
    assert next(iter(sim.grid[1, 1].values())) is extra['agent5']
    sim2 = MultiAgentGridSim.build_sim_from_grid(grid, extra_agents=extra)
    with pytest.raises(AssertionError):
        sim2.reset()                                  # the agents may not overlap
