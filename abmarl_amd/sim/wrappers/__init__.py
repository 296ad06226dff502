from abmarl_amd.sim.wrappers.sar_wrapper import Wrapper, SARWrapper  # noqa: F401
from abmarl_amd.sim.wrappers.ravel_discrete_wrapper import (  # noqa: F401
    RavelDiscreteWrapper, ravel, unravel, ravel_space, check_space)
