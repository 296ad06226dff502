#!/bin/bash
# Round 5: Pacman on the unpadded cell table only -- parity (prod + checks),
# A/B vs HEAD (turn rollouts, per-turn launches), phase stamps.
set -o pipefail
mkdir -p gpurun_out/r05z
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py tests/test_components.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pacman or Pacman or pac" > gpurun_out/r05z/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05z/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05z/tests.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05z/checks.log 2>&1
rc=$?; tail -1 gpurun_out/r05z/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05z/checks.log; exit 1; }
B=abmarl_amd/_build/ab/h4/libgw_engine.so
timeout -k 10 600 bash tools/ab_libs.sh r05z/ab_pac_roll "base=$B new=-" --workload pacman --steps 200 --warmup 5 --fragment 50 --preroll 200 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh r05z/ab_pac_step "base=$B new=-" --workload pacman --mode step --steps 200 --warmup 5 --preroll 200 || exit 1
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps_pac.py > gpurun_out/r05z/stamps_pac.log 2>&1 || { echo STAMPS FAIL; exit 1; }
grep -v amdgpu.ids gpurun_out/r05z/stamps_pac.log
