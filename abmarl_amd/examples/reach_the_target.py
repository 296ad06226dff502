"""ReachTheTarget (reference: abmarl/examples/sim/reach_the_target.py:1-158).

The step program is GW_SIM_REACH_TARGET in the HIP engine:
  attack pass  the target's SelectiveAttackActor attacks, -0.1 on a failed
               attempt, +1 / -1 per kill (:96-108);
  move pass    runners move (-0.1 on failure); a runner on the target's cell
               gets +1, leaves the grid and turns inactive (:110-121) — the
               reference raises KeyError when that runner was already killed
               there by the target (Grid.remove twice); the engine flags
               GW_ERR_DOUBLE_REMOVE and the host raises the same KeyError;
  entropy      -0.01 per runner in the action dict (:123-126).
Dones: runners ActiveDone or TargetDone, the target OnlyAgentLeftDone,
__all__ = OnlyAgentLeftDone (:144-153).  Reset: HealthState, then
PositionState (:88-92).
"""
import numpy as np

from abmarl_amd import _abi
from abmarl_amd.sim.agent_based_simulation import Agent
from abmarl_amd.sim.gridworld.smart import SmartGridWorldSimulation
from abmarl_amd.sim.gridworld.agent import (
    GridWorldAgent, MovingAgent, AttackingAgent, GridObservingAgent, HealthAgent)
from abmarl_amd.sim.gridworld.components import (
    PositionState, HealthState, SelectiveAttackActor, MoveActor, PositionCenteredEncodingObserver,
    ActiveDone, DoneBaseComponent)


class TargetDone(ActiveDone):
    """reach_the_target.py:13-38: an agent is done when it overlaps the target."""
    _program_done = _abi.GW_SIM_REACH_TARGET

    def __init__(self, target=None, **kwargs):
        super().__init__(**kwargs)
        assert target in self.agents.values(), "Target must be an agent."
        self.target = target


class OnlyAgentLeftDone(DoneBaseComponent):
    """reach_the_target.py:41-55: done when at most one active Agent remains."""
    _program_done = _abi.GW_SIM_REACH_TARGET


class BarrierAgent(GridWorldAgent):
    def __init__(self, **kwargs):
        super().__init__(encoding=1, blocking=True, render_shape='s', **kwargs)


class TargetAgent(AttackingAgent, GridObservingAgent):
    def __init__(self, **kwargs):
        super().__init__(id='target', encoding=2, render_color='g', **kwargs)


class RunningAgent(MovingAgent, GridObservingAgent, HealthAgent):
    def __init__(self, **kwargs):
        super().__init__(encoding=3, render_color='b', **kwargs)


class ReachTheTargetSim(SmartGridWorldSimulation):
    _engine_program = _abi.GW_SIM_REACH_TARGET

    def __init__(self, device=None, **kwargs):
        # the reference builds its components explicitly (not from sets) and
        # resets health before positions (:88-92)
        super().__init__(device=device, state_order='health_position', **kwargs)
        self.target = self.agents['target']
        self.position_state = PositionState(**kwargs)
        self.health_state = HealthState(**kwargs)
        self.move_actor = MoveActor(**kwargs)
        self.attack_actor = SelectiveAttackActor(**kwargs)
        self.grid_observer = PositionCenteredEncodingObserver(**kwargs)
        self.active_done = ActiveDone(**kwargs)
        self.target_done = TargetDone(target=self.target, **kwargs)
        self.only_agent_done = OnlyAgentLeftDone(**kwargs)
        self._states = [self.health_state, self.position_state]
        self._observers = [self.grid_observer]
        self._dones = [self.active_done, self.target_done, self.only_agent_done]
        self.finalize()

    def _program_extras(self):
        return dict(target_agent=list(self.agents).index('target'), program_type=RunningAgent)

    def reset(self, **kwargs):
        self._rt().reset()
        self.rewards = {a.id: 0 for a in self.agents.values() if isinstance(a, Agent)}
