"""Simulation wrappers (reference: abmarl/sim/wrappers/wrapper.py:1-52,
sar_wrapper.py:1-58).

A Wrapper is an AgentBasedSimulation around another one: reset/step/get_*
pass through, and `agents` is a deep copy whose spaces the wrapper may
rewrite.  A SARWrapper transforms each agent's observations and rewards on
the way out and its actions on the way in (action: sim <- wrapper <- trainer).
"""
import copy

from abmarl_amd.sim.agent_based_simulation import AgentBasedSimulation


class Wrapper(AgentBasedSimulation):
    def __init__(self, sim):
        assert isinstance(sim, AgentBasedSimulation), \
            "Wrapper can only wrap AgentBasedSimulation."
        self.sim = sim
        self.agents = copy.deepcopy(sim.agents)

    @property
    def unwrapped(self):
        """The innermost simulation."""
        inner = self.sim
        while isinstance(inner, Wrapper):
            inner = inner.sim
        return inner

    def reset(self, **kwargs):
        self.sim.reset(**kwargs)

    def step(self, action_dict, **kwargs):
        self.sim.step(action_dict, **kwargs)

    def render(self, **kwargs):
        self.sim.render(**kwargs)

    def get_obs(self, agent_id, **kwargs):
        return self.sim.get_obs(agent_id, **kwargs)

    def get_reward(self, agent_id, **kwargs):
        return self.sim.get_reward(agent_id, **kwargs)

    def get_done(self, agent_id, **kwargs):
        return self.sim.get_done(agent_id, **kwargs)

    def get_all_done(self, **kwargs):
        return self.sim.get_all_done(**kwargs)

    def get_info(self, agent_id, **kwargs):
        return self.sim.get_info(agent_id, **kwargs)


class SARWrapper(Wrapper):
    def step(self, action_dict, **kwargs):
        self.sim.step({aid: self.wrap_action(self.sim.agents[aid], action)
                       for aid, action in action_dict.items()}, **kwargs)

    def get_obs(self, agent_id, **kwargs):
        return self.wrap_observation(self.sim.agents[agent_id], self.sim.get_obs(agent_id))

    def get_reward(self, agent_id, **kwargs):
        return self.wrap_reward(self.sim.get_reward(agent_id))

    # identity by default; derived wrappers override these
    def wrap_observation(self, from_agent, observation):
        return observation

    def unwrap_observation(self, from_agent, observation):
        return observation

    def wrap_action(self, from_agent, action):
        return action

    def unwrap_action(self, from_agent, action):
        return action

    def wrap_reward(self, reward):
        return reward

    def unwrap_reward(self, reward):
        return reward
