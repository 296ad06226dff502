#!/bin/bash
# Round 5, fault analysis step 2 + HEAD's checks and production suites.
#  1. libgw_probe2_checks.so (95ec8c4 + split pairs + GW_PROBE2: the crossing
#     placements record every lane's key pointer and take the serial path --
#     no flat access through rng.key there): the failing test, then the records;
#  2. HEAD's checks build on the round-4 failing selection + the new tests;
#  3. HEAD's production build: the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
P2=abmarl_amd/_build/fault_r05/libgw_probe2_checks.so
GW_ENGINE_VARIANT=checks GW_ENGINE_LIB=$P2 timeout -k 10 300 python -u -m pytest tests/test_engine_golden.py -x -q \
  --timeout 120 --timeout-method thread -k "test_engine_matches_reference and rtt_16" > gpurun_out/r05b/probe2_test.log 2>&1
rc=$?; tail -2 gpurun_out/r05b/probe2_test.log; [ $rc -eq 0 ] || { echo "PROBE2 TEST rc=$rc"; tail -30 gpurun_out/r05b/probe2_test.log; exit 1; }
GW_ENGINE_VARIANT=checks GW_ENGINE_LIB=$P2 timeout -k 10 120 python -u tools/fault_r05/probe.py rtt_16_example rtt_16 > gpurun_out/r05b/probe2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05b/probe2.log | cut -c1-3000; [ $rc -eq 0 ] || exit 1
SEL="oracle or golden or rollout or components or shard or builders or kernel_resources"
GW_ENGINE_VARIANT=checks timeout -k 10 700 python -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "$SEL" > gpurun_out/r05b/head_checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05b/head_checks.log; [ $rc -eq 0 ] || { echo "HEAD CHECKS rc=$rc"; tail -40 gpurun_out/r05b/head_checks.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05b/head_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05b/head_gpu.log; [ $rc -eq 0 ] || { echo "HEAD GPU rc=$rc"; tail -40 gpurun_out/r05b/head_gpu.log; exit 1; }
