"""AllStepManager (reference: abmarl/managers/all_step_manager.py:8-95).

The control flow is the reference's: reset returns the observation of every
Agent; step asserts that no done agent acts, steps the simulation, then
collects obs, rewards, dones and infos of every agent not yet done (in
agents-dict order), records new dones, and sets '__all__'.  For an
engine-backed GridWorld simulation the simulation's step already computed
all of these in one fused kernel, in this same order, and the getters
return the results; for plain Python simulations (e.g. MultiCorridor) the
getters run as usual.
"""
import random

from abmarl_amd.sim.agent_based_simulation import Agent
from abmarl_amd.managers.simulation_manager import SimulationManager


class AllStepManager(SimulationManager):
    def __init__(self, sim, randomize_action_input=False, **kwargs):
        super().__init__(sim, **kwargs)
        assert type(randomize_action_input) is bool, \
            "Randomize action input must be True or False."
        self.randomize_action_input = randomize_action_input

    def reset(self, **kwargs):
        self.done_agents = set(a.id for a in self.agents.values() if not isinstance(a, Agent))
        self.sim.reset(**kwargs)
        return {a.id: self.sim.get_obs(a.id) for a in self.agents.values()
                if a.id not in self.done_agents}

    def step(self, action_dict, **kwargs):
        for agent_id in action_dict:
            assert agent_id not in self.done_agents, \
                "Received an action for an agent that is already done."
        if self.randomize_action_input:
            items = list(action_dict.items())
            random.shuffle(items)
            action_dict = dict(items)
        self.sim.step(action_dict, **kwargs)
        live = [a.id for a in self.agents.values() if a.id not in self.done_agents]
        obs = {i: self.sim.get_obs(i) for i in live}
        rewards = {i: self.sim.get_reward(i) for i in live}
        dones = {i: self.sim.get_done(i) for i in live}
        infos = {i: self.sim.get_info(i) for i in live}
        for i, d in dones.items():
            if d:
                self.done_agents.add(i)
        dones['__all__'] = bool(self.sim.get_all_done() or
                                not (self.agents.keys() - self.done_agents))
        return obs, rewards, dones, infos
