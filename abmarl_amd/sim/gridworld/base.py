"""GridWorldSimulation builders and the component base class.

Reference: abmarl/sim/gridworld/base.py — build_sim (:38-59),
build_sim_from_grid (:61-96), build_sim_from_array (:98-141),
build_sim_from_file (:143-193), _build_sim (:195-198),
GridWorldBaseComponent (:248-304).  Rendering (:200-245) is out of scope.
"""
from abc import ABC

import numpy as np

from abmarl_amd.sim.agent_based_simulation import AgentBasedSimulation
from abmarl_amd.sim.gridworld.agent import GridWorldAgent
from abmarl_amd.sim.gridworld.grid import Grid


class GridWorldSimulation(AgentBasedSimulation, ABC):
    def __init__(self, grid=None, **kwargs):
        super().__init__(**kwargs)
        self.grid = grid

    @property
    def grid(self):
        return self._grid

    @grid.setter
    def grid(self, value):
        assert isinstance(value, Grid), "Grid must be a Grid object."
        self._grid = value

    @classmethod
    def build_sim(cls, rows, cols, **kwargs):
        assert type(rows) is int, "Rows must be an integer."
        assert 0 < rows, "Rows must be a positive integer."
        assert type(cols) is int, "Cols must be an integer."
        assert 0 < cols, "Cols must be a positive integer."
        return cls._build_sim(rows, cols, **kwargs)

    @classmethod
    def build_sim_from_grid(cls, grid, extra_agents=None, **kwargs):
        """The agents of a Grid's cells, plus extra agents (base.py:61-96).

        An agent found in the grid takes the place of an extra agent with the
        same id (the extra_agents dict is updated in place, as the
        reference's is); every agent in a cell must have that cell as its
        initial position.  The new simulation gets a fresh, empty Grid of the
        same size (placement happens at reset)."""
        assert type(grid) is Grid, "Grid object required."
        if extra_agents is not None:
            assert type(extra_agents) is dict, "Extra agents must be a dictionary."
            agents = extra_agents
        else:
            agents = {}
        for r in range(grid.rows):
            for c in range(grid.cols):
                cell = grid[r, c]
                if cell is None:
                    continue
                agents.update(cell)
                for agent in cell.values():
                    np.testing.assert_array_equal(
                        agent.initial_position, np.array([r, c]),
                        err_msg="The initial position of the agent must match its position in the grid.")
        return cls._build_sim(grid.rows, grid.cols, agents=agents, **kwargs)

    @classmethod
    def build_sim_from_array(cls, array, object_registry, extra_agents=None, **kwargs):
        """Agents from a character array, in row-major order (base.py:98-141)."""
        assert type(array) is np.ndarray, "The array must be a numpy array."
        assert type(object_registry) is dict, "The object_registry must be a dictionary."
        assert all(i not in object_registry for i in [0, '.', '_']), \
            "0, '.', and '_' are reserved for empty space."
        agents = {}
        if extra_agents is not None:
            assert type(extra_agents) is dict, "Extra agents must be a dictionary."
            agents = extra_agents
        n = 0
        for r in range(array.shape[0]):
            for c in range(array.shape[1]):
                ch = array[r, c]
                if ch in object_registry:
                    agent = object_registry[ch](n)
                    agent.initial_position = np.array([r, c])
                    agents[agent.id] = agent
                    n += 1
        return cls._build_sim(array.shape[0], array.shape[1], agents=agents, **kwargs)

    @classmethod
    def build_sim_from_file(cls, file_name, object_registry, extra_agents=None, **kwargs):
        """Space-separated character grid in a text file (base.py:143-193)."""
        assert type(file_name) is str, "The file_name must be the name of the file."
        with open(file_name, 'r') as fp:
            lines = fp.read().splitlines()
        rows = [line.split(' ') for line in lines]
        ncols = len(rows[0])
        for row in rows:
            assert len(row) == ncols, f"Mismatched number of columns per row in {file_name}"
        return cls.build_sim_from_array(np.array(rows, dtype=object), object_registry,
                                        extra_agents=extra_agents, **kwargs)

    @classmethod
    def _build_sim(cls, rows, cols, **kwargs):
        grid = Grid(rows, cols, **kwargs)
        return cls(grid=grid, **kwargs)


class GridWorldBaseComponent(ABC):
    def __init__(self, agents=None, grid=None, **kwargs):
        self.agents = agents
        self.grid = grid

    @property
    def rows(self):
        return self.grid.rows

    @property
    def cols(self):
        return self.grid.cols

    @property
    def grid(self):
        return self._grid

    @grid.setter
    def grid(self, value):
        assert isinstance(value, Grid), "The grid must be a Grid object."
        self._grid = value

    @property
    def agents(self):
        return self._agents

    @agents.setter
    def agents(self, value):
        assert type(value) is dict, "Agents must be a dict."
        for agent_id, agent in value.items():
            assert isinstance(agent, GridWorldAgent), \
                "Values of agents dict must be instance of GridWorldAgent."
            assert agent_id == agent.id, "Keys of agents dict must be the same as the Agent's id."
        self._agents = value
