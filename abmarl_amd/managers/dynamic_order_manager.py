"""DynamicOrderManager (reference: abmarl/managers/dynamic_order_manager.py:6-86).

The simulation names the agent(s) whose turn it is (DynamicOrderSimulation.
next_agent).  reset returns their observations; step refuses actions from
agents already done, steps the simulation, and returns the outputs of the
next agents: an agent that just finished gets its final outputs once and is
recorded as done (the simulation names at least one agent that is not done
unless the episode is over; when every agent is done, __all__ is set).  Once
the simulation reports all done, every agent not yet done gets its outputs.

A host-side protocol: the engine's fused programs run AllStepManager's (or,
for Pacman, TurnBasedManager's) inside their step, so a simulation built on
one of them is refused here.
"""
from abmarl_amd.sim.agent_based_simulation import DynamicOrderSimulation
from abmarl_amd.managers.simulation_manager import SimulationManager


class DynamicOrderManager(SimulationManager):
    def __init__(self, sim, **kwargs):
        assert isinstance(sim, DynamicOrderSimulation), \
            "DynamicOrderManager needs a DynamicOrderSimulation."
        if getattr(sim, '_engine_program', None) is not None:
            raise NotImplementedError(
                f"{type(sim).__name__} runs a fused manager protocol on the engine; the dynamic-order "
                "protocol is for host-side simulations")
        super().__init__(sim, **kwargs)

    def reset(self, **kwargs):
        self.done_agents = set()
        self.sim.reset(**kwargs)
        return {aid: self.sim.get_obs(aid) for aid in self.sim.next_agent}

    def _collect(self, aid, out):
        obs, rewards, dones, infos = out
        obs[aid] = self.sim.get_obs(aid)
        rewards[aid] = self.sim.get_reward(aid)
        dones[aid] = self.sim.get_done(aid)
        infos[aid] = self.sim.get_info(aid)

    def step(self, action_dict, **kwargs):
        assert not any(aid in self.done_agents for aid in action_dict), \
            "Received an action for an agent that is already done."
        self.sim.step(action_dict, **kwargs)
        out = ({}, {}, {'__all__': self.sim.get_all_done()}, {})
        if out[2]['__all__']:
            for aid in self.agents:
                if aid not in self.done_agents:
                    self._collect(aid, out)
            return out
        for aid in self.sim.next_agent:
            if aid in self.done_agents:
                continue                                  # no interaction with it any more
            self._collect(aid, out)
            if out[2][aid]:
                # just finished: its final outputs go out this once
                self.done_agents.add(aid)
                if all(a in self.done_agents for a in self.agents):
                    out[2]['__all__'] = True
                    break
        return out
