#!/bin/bash
# Round 5: the Lehmer-decode placement (shared list) -- GPU suite, stamps, A/B.
set -o pipefail
mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05g/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 gpurun_out/r05g/gpu.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r05g/stamps_tb.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r05g/stamps_tb.log; exit 1; }
timeout -k 10 900 bash tools/ab_libs.sh r05g/ab_lehmer "base=abmarl_amd/_build/ab/base/libgw_engine.so:0 new=-:0 base_r=abmarl_amd/_build/ab/base/libgw_engine.so:-1 new_r=-:-1" || exit 1
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or oracle or rollout" > gpurun_out/r05g/checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05g/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -40 gpurun_out/r05g/checks.log; exit 1; }
