"""Agent classes and the AgentBasedSimulation interface.

Same names, attributes and assertion behaviour as the reference's
abmarl/sim/agent_based_simulation.py (PrincipleAgent :7-63, ActingAgent :66-117,
ObservingAgent :120-171, Agent :174-186, AgentBasedSimulation :189-294).
"""
from abc import ABC, abstractmethod
from collections.abc import Container

from abmarl_amd import spaces as sp
from abmarl_amd.sim import host_version


class PrincipleAgent:
    def __init__(self, id=None, seed=None, **kwargs):
        self.id = id
        self.seed = seed
        self.active = True

    @property
    def id(self):
        return self._id

    @id.setter
    def id(self, value):
        assert type(value) is str, "id must be a string."
        self._id = value

    @property
    def seed(self):
        return self._seed

    @seed.setter
    def seed(self, value):
        assert value is None or type(value) is int, "Seed must be an integer."
        self._seed = value

    @property
    def active(self):
        return self._active

    @active.setter
    def active(self, value):
        assert type(value) is bool, "Active must be either True or False."
        self._active = value
        host_version.bump()

    @property
    def configured(self):
        return self.id is not None

    def finalize(self, **kwargs):
        pass

    def __eq__(self, other):
        return isinstance(other, self.__class__) and self.__dict__ == other.__dict__


class ActingAgent(PrincipleAgent):
    def __init__(self, action_space=None, null_action=None, **kwargs):
        super().__init__(**kwargs)
        self.action_space = action_space
        self.null_action = null_action

    @property
    def action_space(self):
        return self._action_space

    @action_space.setter
    def action_space(self, value):
        assert value is None or sp.check_space(value), \
            "The action space must be None, a Space, or a dict of Spaces."
        self._action_space = {} if value is None else value

    @property
    def null_action(self):
        return self._null_action

    @null_action.setter
    def null_action(self, value):
        self._null_action = {} if value is None else value

    @property
    def configured(self):
        return super().configured and sp.check_space(self.action_space, strict=True)

    def finalize(self, **kwargs):
        super().finalize(**kwargs)
        if type(self.action_space) is dict:
            self.action_space = sp.make_dict(self.action_space)
        self.action_space.seed(self.seed)


class ObservingAgent(PrincipleAgent):
    def __init__(self, observation_space=None, null_observation=None, **kwargs):
        super().__init__(**kwargs)
        self.observation_space = observation_space
        self.null_observation = null_observation

    @property
    def observation_space(self):
        return self._observation_space

    @observation_space.setter
    def observation_space(self, value):
        assert value is None or sp.check_space(value), \
            "The observation space must be None, a Space, or a dict of Spaces."
        self._observation_space = {} if value is None else value

    @property
    def null_observation(self):
        return self._null_observation

    @null_observation.setter
    def null_observation(self, value):
        self._null_observation = {} if value is None else value

    @property
    def configured(self):
        return super().configured and sp.check_space(self.observation_space, strict=True)

    def finalize(self, **kwargs):
        super().finalize(**kwargs)
        if type(self.observation_space) is dict:
            self.observation_space = sp.make_dict(self.observation_space)
        self.observation_space.seed(self.seed)


class _AgentMeta(type):
    def __instancecheck__(cls, instance):
        return isinstance(instance, ObservingAgent) and isinstance(instance, ActingAgent)


class Agent(ObservingAgent, ActingAgent, metaclass=_AgentMeta):
    """An agent that both observes and acts (the reference's AgentMeta check)."""


class AgentBasedSimulation(ABC):
    def __init__(self, agents=None, **kwargs):
        self.agents = agents

    @property
    def agents(self):
        return self._agents

    @agents.setter
    def agents(self, value):
        assert type(value) is dict, "Agents must be a dict."
        for agent_id, agent in value.items():
            assert isinstance(agent, PrincipleAgent), \
                "Values of agents dict must be instance of PrincipleAgent."
            assert agent_id == agent.id, "Keys of agents dict must be the same as the Agent's id."
        self._agents = value

    def finalize(self):
        for agent in self.agents.values():
            agent.finalize()
            assert agent.configured

    @abstractmethod
    def reset(self, **kwargs):
        pass

    @abstractmethod
    def step(self, action, **kwargs):
        pass

    def render(self, **kwargs):
        raise NotImplementedError("Rendering is outside the engine's scope.")

    @abstractmethod
    def get_obs(self, agent_id, **kwargs):
        pass

    @abstractmethod
    def get_reward(self, agent_id, **kwargs):
        pass

    @abstractmethod
    def get_done(self, agent_id, **kwargs):
        pass

    @abstractmethod
    def get_all_done(self, **kwargs):
        pass

    @abstractmethod
    def get_info(self, agent_id, **kwargs):
        pass


class DynamicOrderSimulation(AgentBasedSimulation):
    """A simulation that decides whose turn comes next as it runs
    (reference: abmarl/sim/agent_based_simulation.py:297-317): next_agent is
    one agent id or a container of them, every one an agent of the sim; a
    single id is held as a one-element list."""

    @property
    def next_agent(self):
        return self._next_agent

    @next_agent.setter
    def next_agent(self, value):
        assert isinstance(value, (str, Container)), \
            "next_agent takes an agent id or a container of agent ids."
        ids = [value] if type(value) is str else value
        assert all(aid in self.agents for aid in ids), \
            "Each next agent must be one of the simulation's agents."
        self._next_agent = ids
