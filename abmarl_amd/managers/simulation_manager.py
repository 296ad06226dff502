"""SimulationManager (reference: abmarl/managers/simulation_manager.py:6-56)."""
from abc import ABC, abstractmethod

from abmarl_amd.sim.agent_based_simulation import AgentBasedSimulation


class SimulationManager(ABC):
    def __init__(self, sim, **kwargs):
        assert isinstance(sim, AgentBasedSimulation), \
            "SimulationManager can only interface with AgentBasedSimulation."
        self.sim = sim
        self.agents = sim.agents
        self.done_agents = set()

    @abstractmethod
    def reset(self, **kwargs):
        pass

    @abstractmethod
    def step(self, action_dict, **kwargs):
        pass

    def render(self, **kwargs):
        self.sim.render(**kwargs)
