"""Known answers for PositionState(randomize_placement_order=True) from the
REFERENCE (run in this container; needs /root/reference): six resets of a
2x3 grid after random.seed(3), np.random.seed(5).  The printed lists are the
data in tests/test_components.py::test_position_state_randomize_placement_order.
"""
import os
import sys, random
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gym_stub
gym_stub.install()
sys.path.insert(0, '/root/reference')
from abmarl.sim.gridworld.grid import Grid
from abmarl.sim.gridworld.agent import GridWorldAgent
from abmarl.sim.gridworld.state import PositionState
agents = {'a0': GridWorldAgent(id='a0', encoding=1), 'a1': GridWorldAgent(id='a1', encoding=2),
          'a2': GridWorldAgent(id='a2', encoding=1, initial_position=np.array([0, 0])),
          'a3': GridWorldAgent(id='a3', encoding=2), 'a4': GridWorldAgent(id='a4', encoding=1)}
grid = Grid(2, 3, overlapping={1: {1}})
state = PositionState(grid=grid, agents=agents, randomize_placement_order=True)
random.seed(3); np.random.seed(5)
out = []
for _ in range(6):
    state.reset()
    out.append([list(map(int, agents[k].position)) for k in ['a0', 'a1', 'a2', 'a3', 'a4']] +
               [[k for k in grid[0, 0]]])
print(out)
print(np.random.get_state()[2], random.random())
