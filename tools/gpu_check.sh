#!/bin/bash
# GPU round: [checks-build tests], tests, bench, [probe], [stamps]; each step
# time-limited, stop at the first failure.
#   tools/gpu_check.sh [checks] [probe] [stamps] [nobench]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=" $* "
if [[ "$ARGS" == *" checks "* ]]; then
  GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_checks.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests_checks.log
  [ $rc -eq 0 ] || { echo "CHECKS TESTS FAILED rc=$rc"; tail -60 gpurun_out/gpu_tests_checks.log; exit 1; }
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
if [[ "$ARGS" != *" nobench "* ]]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/bench20.log 2>&1 || { echo BENCH20 FAIL; tail -30 gpurun_out/bench20.log; exit 1; }
  tail -1 gpurun_out/bench20.log
fi
if [[ "$ARGS" == *" probe "* ]]; then
  timeout -k 10 120 python tools/graph_probe.py > gpurun_out/probe.log 2>&1 || { echo PROBE FAIL; tail -20 gpurun_out/probe.log; exit 1; }
  tail -1 gpurun_out/probe.log
fi
if [[ "$ARGS" == *" stamps "* ]]; then
  MODE=${MODE:-same_step} HORIZON=${HORIZON:-100000} timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/stamps.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps.log
fi
