#!/bin/bash
# Round 5: Pacman observation walk (branch-free) -- parity, A/B (turn rollouts
# and per-turn launches), phase stamps.
set -o pipefail
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05m/pac_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05m/pac_tests.log; [ $rc -eq 0 ] || { echo "PAC rc=$rc"; tail -40 gpurun_out/r05m/pac_tests.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05m/pac_checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05m/pac_checks.log; [ $rc -eq 0 ] || { echo "PAC CHECKS rc=$rc"; tail -40 gpurun_out/r05m/pac_checks.log; exit 1; }
B=abmarl_amd/_build/ab/base/libgw_engine.so
timeout -k 10 600 bash tools/ab_libs.sh r05m/ab_pac_roll "base=$B new=-" --workload pacman --steps 200 --warmup 5 --fragment 50 --preroll 200 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh r05m/ab_pac_step "base=$B new=-" --workload pacman --mode step --steps 200 --warmup 5 --preroll 200 || exit 1
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps_pac.py > gpurun_out/r05m/stamps_pac.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r05m/stamps_pac.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05m/stamps_pac.log
