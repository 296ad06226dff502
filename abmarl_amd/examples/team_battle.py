"""TeamBattle (reference: abmarl/examples/sim/team_battle_example.py:11-59).

The step program (attack pass -> move pass -> entropy penalty, rewards
-0.1 failed attack, +1/-1 per kill, -0.1 failed move, -0.01 per acting agent)
is GW_SIM_TEAM_BATTLE in the HIP engine.
"""
from abmarl_amd import _abi
from abmarl_amd.sim.gridworld.smart import SmartGridWorldSimulation
from abmarl_amd.sim.gridworld.agent import (
    GridObservingAgent, MovingAgent, AttackingAgent, HealthAgent)
from abmarl_amd.sim.gridworld.components import MoveActor, BinaryAttackActor


class BattleAgent(GridObservingAgent, MovingAgent, AttackingAgent, HealthAgent):
    def __init__(self, **kwargs):
        super().__init__(move_range=1, attack_range=1, attack_strength=1, attack_accuracy=1,
                         view_range=3, **kwargs)


class TeamBattleSim(SmartGridWorldSimulation):
    _engine_program = _abi.GW_SIM_TEAM_BATTLE

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.move_actor = MoveActor(**kwargs)
        self.attack_actor = BinaryAttackActor(**kwargs)
        self.finalize()
