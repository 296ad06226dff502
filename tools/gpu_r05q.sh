#!/bin/bash
# Round 5: headline A/B round 4's final build vs HEAD (same box); Pacman A/B
# HEAD-committed vs the full-grid walk vs + action prefetch; Pacman tests.
set -o pipefail
mkdir -p gpurun_out/r05q
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05q/pac_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05q/pac_tests.log; [ $rc -eq 0 ] || { echo "PAC rc=$rc"; tail -30 gpurun_out/r05q/pac_tests.log; exit 1; }
GW_ENGINE_LIB=abmarl_amd/_build/ab/pref/libgw_engine.so timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05q/pac_tests_pref.log 2>&1
rc=$?; tail -1 gpurun_out/r05q/pac_tests_pref.log; [ $rc -eq 0 ] || { echo "PAC PREF rc=$rc"; tail -30 gpurun_out/r05q/pac_tests_pref.log; exit 1; }
R4=abmarl_amd/_build/ab/r04/libgw_engine.so
B=abmarl_amd/_build/ab/base/libgw_engine.so
P=abmarl_amd/_build/ab/pref/libgw_engine.so
timeout -k 10 600 bash tools/ab_libs.sh r05q/ab_headline "r04=$R4 head=-" --steps 20 --warmup 5 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh r05q/ab_pac_roll "base=$B full=- pref=$P" --workload pacman --steps 200 --warmup 5 --fragment 50 --preroll 200 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh r05q/ab_pac_step "base=$B full=- pref=$P" --workload pacman --mode step --steps 200 --warmup 5 --preroll 200 || exit 1
