"""The benchmark workloads of BASELINE.json, built with the package's own
host API (no test fixtures): bench.py and the parity tests share them.

  team_battle_sim  configs[2] (the metric's config): TeamBattle 32x32, 64
                   BattleAgents in 2 teams (team_battle_example.py:11-59)
  maze_sim         configs[1]: MazeNavigation 16x16, one navigator, blocking
                   walls (rllib_maze_navigation.py); the map is MAZE_16
  rtt_sim          configs[3]: ReachTheTarget 64x64, 128 barriers + 127
                   runners + the target in the center (256 entities,
                   rllib_reach_the_target.py's agent parameters)
  pacman_sim       configs[4]: pacman.txt with four baddies
"""
import numpy as np

from abmarl_amd.examples.team_battle import BattleAgent, TeamBattleSim
from abmarl_amd.examples.maze_navigation import MazeNavigationAgent, MazeNavigationSim
from abmarl_amd.examples.reach_the_target import (
    ReachTheTargetSim, RunningAgent, TargetAgent, BarrierAgent)
from abmarl_amd.sim.gridworld.agent import GridWorldAgent

# A 16x16 maze drawn by the reference's generate_maze (utils.py:120-212),
# seed 9 (the maze_16 parity fixture's map): N navigator, T target, W wall.
MAZE_16 = (
    'N__TW_______W_W_',
    'WW_W_WWWW_W_____',
    '_W_W__W__WW_WW_W',
    '_W__W_WW_W___W_W',
    '__W_W_W____W__W_',
    'W______WWW__W___',
    'WW_W_W__W__W_W_W',
    'WWW__WW__W____W_',
    'WWWW__WW___W_WW_',
    'WWWW_WW__W_W____',
    'WWW__W__W_WWWWW_',
    'WW__W_W________W',
    'W__WW__W_WW_W_W_',
    '_WWW_W____W_W___',
    '_______W_WW__W_W',
    'W_W_W_W___W_W___',
)


def team_battle_sim(rows=32, cols=32, n_agents=64, n_teams=2):
    """TeamBattle as in team_battle_example.py:62-80 with BASELINE's sizes."""
    agents = {f'agent{i}': BattleAgent(id=f'agent{i}', encoding=i % n_teams + 1)
              for i in range(n_agents)}
    return TeamBattleSim.build_sim(
        rows, cols, agents=agents,
        overlapping={t: {t} for t in range(1, n_teams + 1)},
        attack_mapping={t: {u for u in range(1, n_teams + 1) if u != t}
                        for t in range(1, n_teams + 1)},
        states={'PositionState', 'HealthState'},
        observers={'PositionCenteredEncodingObserver'},
        dones={'OneTeamRemainingDone'})


def maze_sim(maze=MAZE_16, view_range=2):
    """MazeNavigation from a maze array (rllib_maze_navigation.py's registry)."""
    registry = {
        'N': lambda n: MazeNavigationAgent(id='navigator', encoding=1, view_range=view_range),
        'T': lambda n: GridWorldAgent(id='target', encoding=3),
        'W': lambda n: GridWorldAgent(id=f'wall{n}', encoding=2, blocking=True),
    }
    arr = np.array([list(r) for r in maze], dtype=object)
    return MazeNavigationSim.build_sim_from_array(
        arr, registry, overlapping={1: {3}, 3: {1}},
        states={'PositionState'}, observers={'PositionCenteredEncodingObserver'})


def rtt_sim(rows=64, cols=64, n_barriers=128, n_runners=127):
    """ReachTheTarget with rllib_reach_the_target.py's agent parameters
    (runners: move 2, view 3, health 1; target: view 3, attack 1, strength 1,
    accuracy 1) and the target in the center."""
    agents = {f'barrier{i}': BarrierAgent(id=f'barrier{i}') for i in range(n_barriers)}
    for i in range(n_runners):
        agents[f'runner{i}'] = RunningAgent(id=f'runner{i}', move_range=2, view_range=3,
                                            initial_health=1)
    agents['target'] = TargetAgent(view_range=3, attack_range=1, attack_strength=1,
                                   attack_accuracy=1,
                                   initial_position=np.array([rows // 2, cols // 2], dtype=int))
    return ReachTheTargetSim.build_sim(rows, cols, agents=agents,
                                       overlapping={2: {3}, 3: {1, 2, 3}}, attack_mapping={2: {3}})


def pacman_sim():
    """pacman.txt with four baddies (BASELINE config 5)."""
    from abmarl_amd.examples.pacman import build_pacman
    return build_pacman()
