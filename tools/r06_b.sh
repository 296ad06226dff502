#!/bin/bash
# Round 6, step B: rocprofv3 kernel-trace + PMC evidence (tools/prof_headline.sh)
# for config 4's timed 100-step launch (1024 envs, one dispatch round now),
# config 5's timed 50-turn gw_turn_rollout launch, and the headline's timed
# 20-step launch: gpurun_out/ph_<tag>/
set -o pipefail
export TMPDIR=/tmp
for W in "r06rtt rtt" "r06pac pacman" "r06tb team_battle"; do
  set -- $W
  timeout -k 10 1000 bash tools/prof_headline.sh $1 $2 > gpurun_out/prof_$1.log 2>&1 || { echo "PROF $1 FAIL"; tail -30 gpurun_out/prof_$1.log; exit 1; }
  tail -n 25 gpurun_out/prof_$1.log
done
