#!/bin/bash
# Round 5: config 4's crowded draws with three barriers fewer and a
# double-buffered offset scan: parity (prod + checks), A/B vs HEAD, stamps.
set -o pipefail
mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "reach_the_target or rtt or workgroup or golden" > gpurun_out/r05t/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05t/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05t/tests.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "reach_the_target or rtt_" > gpurun_out/r05t/checks.log 2>&1
rc=$?; tail -1 gpurun_out/r05t/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05t/checks.log; exit 1; }
timeout -k 10 900 bash tools/ab_libs.sh r05t/ab_rtt "base=abmarl_amd/_build/ab/c4base/libgw_engine.so new=-" --workload rtt --steps 100 --warmup 5 || exit 1
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r05t/stamps_rtt.log 2>&1 || { echo STAMPS FAIL; exit 1; }
grep -v amdgpu.ids gpurun_out/r05t/stamps_rtt.log | tail -8
