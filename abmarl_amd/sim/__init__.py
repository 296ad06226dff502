from abmarl_amd.sim.agent_based_simulation import (  # noqa: F401
    PrincipleAgent, ActingAgent, ObservingAgent, Agent, AgentBasedSimulation, DynamicOrderSimulation)
