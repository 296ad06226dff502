"""MazeNavigation (reference: abmarl/examples/sim/maze_navigation.py:8-42).

The step program (move the navigator, -0.1 on a failed move, +1 when it
stands on the target, -0.01 entropy; done = navigator on target) is
GW_SIM_MAZE_NAV in the HIP engine.  Walls built from a maze array or file
(examples/rllib_maze_navigation.py) are static blocking entities of the
engine: they hide cells from the navigator's view (utils.py:46-115).
"""
from abmarl_amd import _abi
from abmarl_amd.sim.gridworld.smart import SmartGridWorldSimulation
from abmarl_amd.sim.gridworld.agent import GridObservingAgent, MovingAgent
from abmarl_amd.sim.gridworld.components import MoveActor


class MazeNavigationAgent(GridObservingAgent, MovingAgent):
    def __init__(self, **kwargs):
        super().__init__(move_range=1, **kwargs)


class MazeNavigationSim(SmartGridWorldSimulation):
    _engine_program = _abi.GW_SIM_MAZE_NAV

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.navigator = self.agents['navigator']
        self.target = self.agents['target']
        self.move_actor = MoveActor(**kwargs)
        self.finalize()

    def _program_extras(self):
        ids = list(self.agents)
        return dict(nav_agent=ids.index('navigator'), target_agent=ids.index('target'))

    # maze_navigation.py:38-42 (no done components: the sim decides)
    def get_done(self, agent_id, **kwargs):
        return self._rt().get_done(agent_id)

    def get_all_done(self, **kwargs):
        return self._rt().get_all_done()
