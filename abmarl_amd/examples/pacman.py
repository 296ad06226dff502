"""Pacman (reference: abmarl/examples/sim/pacman.py:1-158, examples/pacman.txt,
examples/rllib_pacman.py).

The step program is GW_SIM_PACMAN in the HIP engine:
  pacman     DriftMoveActor move (entropy reward when it moves, bad_move when
             it cannot), the tunnel (9,0) <-> (9,20), then the overlaps on its
             cell: food is eaten (eat_food, removed, health 0), a baddie there
             kills it (pacman die, baddie kill) (:80-105);
  baddies    each in the action dict: drift move, reward, tunnel (:107-113);
  overlaps   once more on pacman's cell, baddies only (:115-122); a dead
             pacman leaves the grid (:126-127).
get_done(agent) = get_all_done = pacman is dead (eaten food stays in the
agents dict, so the "no food left" branch of :141-153 never fires while the
map has food).

Turn-based play.  The reference's PacmanSim.step reads action_dict['pacman']
unconditionally, so under TurnBasedManager it raises KeyError on the first
baddie turn.  The engine's program runs pacman's part only when
pacman is in the action dict and each baddie's part only when that baddie is:
under AllStepManager (every live agent in the dict) this is exactly the
reference; under TurnBasedManager it is the build-defined turn-based Pacman
of BASELINE config 5.
"""
import numpy as np

from abmarl_amd import _abi
from abmarl_amd.sim.agent_based_simulation import Agent
from abmarl_amd.sim.gridworld.smart import SmartGridWorldSimulation
from abmarl_amd.sim.gridworld.agent import (
    MovingAgent, OrientationAgent, GridWorldAgent, GridObservingAgent, HealthAgent)
from abmarl_amd.sim.gridworld.components import DriftMoveActor


class PacmanAgent(MovingAgent, OrientationAgent, GridObservingAgent, HealthAgent):
    def __init__(self, **kwargs):
        super().__init__(move_range=1, view_range=100, initial_health=1, **kwargs)


class WallAgent(GridWorldAgent):
    pass


class FoodAgent(HealthAgent):
    def __init__(self, **kwargs):
        super().__init__(render_size=50, initial_health=1, **kwargs)


class BaddieAgent(MovingAgent, OrientationAgent, GridObservingAgent):
    def __init__(self, **kwargs):
        super().__init__(move_range=1, view_range=100, **kwargs)


REWARD_EVENTS = ('bad_move', 'entropy', 'eat_food', 'kill', 'die')


class PacmanSim(SmartGridWorldSimulation):
    """pacman.py:29-158.  State components are pinned to the order
    PositionState, OrientationState, HealthState (only OrientationState
    draws when every HealthAgent has an initial health)."""
    _engine_program = _abi.GW_SIM_PACMAN
    tunnel = (9, 0, 9, 20)                     # hard-coded in pacman.py:88-93

    def __init__(self, reward_scheme=None, **kwargs):
        super().__init__(**kwargs)
        self.pacman = self.agents['pacman']
        self.move_actor = DriftMoveActor(**kwargs)
        self.reward_scheme = reward_scheme
        self.finalize()

    @property
    def reward_scheme(self):
        return self._reward_scheme

    @reward_scheme.setter
    def reward_scheme(self, value):
        if value is not None:
            assert type(value) is dict, "Reward scheme must be a dictionary."
            for event, reward in value.items():
                assert event in REWARD_EVENTS, \
                    "Supported events: 'bad_move', 'entropy', 'eat_food', 'kill', and 'die'."
                assert type(reward) in [int, float], f"Reward for {event} must be numerical."
            # events missing from a user scheme raise KeyError in the reference
            # when they happen; the engine needs a value, so they must be given
            missing = [e for e in REWARD_EVENTS if e not in value]
            assert not missing, f"reward_scheme needs every event; missing {missing}"
            self._reward_scheme = value
        else:
            self._reward_scheme = {'bad_move': -0.1, 'entropy': 0.01, 'eat_food': 0.1,
                                   'kill': 1, 'die': -1}

    def _program_extras(self):
        ids = list(self.agents)
        return dict(pacman_agent=ids.index('pacman'), program_type=BaddieAgent,
                    food_type=FoodAgent, tunnel=self.tunnel,
                    pac_rewards=tuple(float(self.reward_scheme[e]) for e in REWARD_EVENTS))

    def reset(self, **kwargs):
        self._rt().reset()
        self.rewards = {a.id: 0 for a in self.agents.values() if isinstance(a, Agent)}

    # pacman.py:138-153 (no done components: the sim decides)
    def get_done(self, agent_id, **kwargs):
        return self._rt().get_all_done()

    def get_all_done(self, **kwargs):
        return self._rt().get_all_done()


# examples/pacman.txt: P pacman, W wall, F food, B baddie, _ empty
PACMAN_MAP = """
_WWWWWWWWWWWWWWWWWWW_
_WBFFFFFFFWFFFFFFFBW_
_WFWWFWWWFWFWWWFWWFW_
_WFFFFFFFFFFFFFFFFFW_
_WFWWFWFWWWWWFWFWWFW_
_WFFFFWFFFWFFFWFFFFW_
_WWWWFWWW_W_WWWFWWWW_
____WFW_______WFW____
WWWWWFW_WWFWW_WFWWWWW
_____B__BFBFB__B_____
WWWWWFW_WWFWW_WFWWWWW
____WFW_______WFW____
_WWWWFW_WWWWW_WFWWWW_
_WBFFFFFFFWFFFFFFFBW_
_WFWWFWWWFWFWWWFWWFW_
_WFFWFFFFFPFFFFFWFFW_
_WWFWFWFWWWWWFWFWFWW_
_WFFFFWFFFWFFFWFFFFW_
_WFWWWWWWFWFWWWWWWFW_
_WFFFFFFFFBFFFFFFFFW_
_WWWWWWWWWWWWWWWWWWW_
"""

# BASELINE config 5 keeps four baddies: the ghost-house row (9, *) minus the
# one at (9, 15); the other 'B' cells become empty
CONFIG5_BADDIES = ((9, 5), (9, 8), (9, 10), (9, 12))


def pacman_grid(baddies=None):
    """The pacman.txt array; `baddies` (cells) keeps only those 'B' cells."""
    rows = [list(line) for line in PACMAN_MAP.strip().splitlines()]
    arr = np.array(rows, dtype=object)
    if baddies is not None:
        keep = {tuple(b) for b in baddies}
        for r, c in zip(*np.nonzero(arr == 'B')):
            if (int(r), int(c)) not in keep:
                arr[r, c] = '_'
    return arr


def object_registry():
    """examples/rllib_pacman.py:8-33 (render attributes dropped)."""
    return {
        'P': lambda n: PacmanAgent(id='pacman', encoding=1),
        'W': lambda n: WallAgent(id=f'wall_{n}', encoding=2),
        'F': lambda n: FoodAgent(id=f'food_{n}', encoding=3),
        'B': lambda n: BaddieAgent(id=f'baddie_{n}', encoding=4),
    }


def build_pacman(baddies=CONFIG5_BADDIES, reward_scheme=None, **kwargs):
    """PacmanSim on pacman.txt as examples/rllib_pacman.py configures it
    (overlapping {1: {3, 4}, 4: {3, 4}}, AbsoluteEncodingObserver)."""
    return PacmanSim.build_sim_from_array(
        pacman_grid(baddies), object_registry(),
        states={'PositionState', 'OrientationState', 'HealthState'},
        observers={'AbsoluteEncodingObserver'}, overlapping={1: {3, 4}, 4: {3, 4}},
        reward_scheme=reward_scheme, **kwargs)
