#!/bin/bash
# Round 5: next-step actions loaded a step ahead in the one-wave kernel
# (GW_ACT_AHEAD=1 build) -- parity, A/B on the driver's command and 100-step
# fragments; the Pacman two-foods refusal test on HEAD.
set -o pipefail
mkdir -p gpurun_out/r05y
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -k two_foods > gpurun_out/r05y/refuse.log 2>&1
rc=$?; tail -1 gpurun_out/r05y/refuse.log; [ $rc -eq 0 ] || { echo "REFUSE rc=$rc"; tail -30 gpurun_out/r05y/refuse.log; exit 1; }
L=abmarl_amd/_build/ab/ahead/libgw_engine.so
GW_ENGINE_LIB=$L timeout -k 10 900 python -u -m pytest tests/test_rollout.py tests/test_engine_oracle.py tests/test_shard_engine.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rollout or timed_launch or shard or headline" > gpurun_out/r05y/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05y/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05y/tests.log; exit 1; }
timeout -k 10 900 bash tools/ab_libs.sh r05y/ab_headline "head=- ahead=$L" || exit 1
timeout -k 10 900 bash tools/ab_libs.sh r05y/ab_f100 "head=- ahead=$L" --steps 300 --warmup 5 || exit 1
