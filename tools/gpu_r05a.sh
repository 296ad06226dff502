#!/bin/bash
# Round 5, fault root cause + the fix (DESIGN §4 "MT19937 key addressing"):
#  1. 95ec8c4's checks build with its key[i]/key[i+1] pairs split into dword
#     loads (tools/fault_r05/make_variants.py `split`), the round-4 failing test
#     selection, then the GW_PROBE records;
#  2. HEAD's checks build, the same selection + the generic-window twist test.
set -o pipefail
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
SEL="oracle or golden or rollout or components or shard or builders"
SPLIT=abmarl_amd/_build/fault_r05/libgw_split_checks.so
GW_ENGINE_VARIANT=checks GW_ENGINE_LIB=$SPLIT timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "$SEL" > gpurun_out/r05a/split_checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05a/split_checks.log; [ $rc -eq 0 ] || { echo "SPLIT rc=$rc"; tail -40 gpurun_out/r05a/split_checks.log; exit 1; }
GW_ENGINE_VARIANT=checks GW_ENGINE_LIB=$SPLIT timeout -k 10 120 python -u tools/fault_r05/probe.py > gpurun_out/r05a/split_probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05a/split_probe.log; [ $rc -eq 0 ] || exit 1
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "$SEL" > gpurun_out/r05a/head_checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05a/head_checks.log; [ $rc -eq 0 ] || { echo "HEAD CHECKS rc=$rc"; tail -40 gpurun_out/r05a/head_checks.log; exit 1; }
# 3. HEAD's production build: the whole GPU suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05a/head_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05a/head_gpu.log; [ $rc -eq 0 ] || { echo "HEAD GPU rc=$rc"; tail -40 gpurun_out/r05a/head_gpu.log; exit 1; }
