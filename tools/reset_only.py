"""Diagnostic workload: gw_reset on every env, repeated (for rocprofv3 PMC)."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from abmarl_amd.engine import GridWorldEngine, env_seeds  # noqa: E402

cc = bench.team_battle_sim().compiled()
E = int(os.environ.get('ENVS', '4096'))
eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
for i in range(int(os.environ.get('REPS', '20'))):
    eng.reset()
torch.cuda.synchronize()
print("done")
