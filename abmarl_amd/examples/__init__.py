from abmarl_amd.examples.team_battle import BattleAgent, TeamBattleSim  # noqa: F401
from abmarl_amd.examples.multi_corridor import MultiCorridor  # noqa: F401
from abmarl_amd.examples.maze_navigation import MazeNavigationAgent, MazeNavigationSim  # noqa: F401
from abmarl_amd.examples.reach_the_target import (  # noqa: F401
    ReachTheTargetSim, RunningAgent, TargetAgent, BarrierAgent, TargetDone, OnlyAgentLeftDone)
from abmarl_amd.examples.traffic_corridor import (  # noqa: F401
    TrafficCorridorSimulation, TrafficAgent, WallAgent, TargetAgent as TrafficTargetAgent)
