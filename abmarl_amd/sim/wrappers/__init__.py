from abmarl_amd.sim.wrappers.sar_wrapper import Wrapper, SARWrapper  # noqa: F401
from abmarl_amd.sim.wrappers.ravel_discrete_wrapper import (  # noqa: F401
    RavelDiscreteWrapper, ravel, unravel, ravel_space, check_space)
from abmarl_amd.sim.wrappers.flatten_wrapper import (  # noqa: F401
    FlattenWrapper, FlattenActionWrapper, flatten, unflatten, flatten_space, flatdim)
from abmarl_amd.sim.wrappers.super_agent_wrapper import (  # noqa: F401
    SuperAgentWrapper, BatchedSuperAgents)
