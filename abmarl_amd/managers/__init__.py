from abmarl_amd.managers.simulation_manager import SimulationManager  # noqa: F401
from abmarl_amd.managers.all_step_manager import AllStepManager  # noqa: F401
from abmarl_amd.managers.turn_based_manager import TurnBasedManager  # noqa: F401
from abmarl_amd.managers.dynamic_order_manager import DynamicOrderManager  # noqa: F401
