#!/bin/bash
# Round 5 HEAD (reset weight 384, placement confirm check): the whole GPU suite, smoke, the driver's command.
set -o pipefail
mkdir -p gpurun_out/r05fin3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05fin3/gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05fin3/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 gpurun_out/r05fin3/gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05fin3/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r05fin3/smoke.log; exit 1; }
tail -1 gpurun_out/r05fin3/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05fin3/bench_driver.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r05fin3/bench_driver.log; exit 1; }
tail -1 gpurun_out/r05fin3/bench_driver.log | cut -c1-600
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05fin3/checks.log 2>&1
rc=$?; tail -n1 gpurun_out/r05fin3/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05fin3/checks.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r05fin3/stamps_tb.log 2>&1 || { echo STAMPS FAIL; exit 1; }
grep -E 'placement|jacobi' gpurun_out/r05fin3/stamps_tb.log
