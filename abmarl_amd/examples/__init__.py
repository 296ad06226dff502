from abmarl_amd.examples.team_battle import BattleAgent, TeamBattleSim  # noqa: F401
