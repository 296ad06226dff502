#!/bin/bash
# Round 5 final HEAD: the GPU suite, checks build, smoke, the driver's command,
# config 4's rocprof evidence.
set -o pipefail
mkdir -p gpurun_out/r05fin4
export TMPDIR=/tmp
A=abmarl_amd/_build/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05fin4/gpu.log 2>&1
rc=$?; tail -n1 gpurun_out/r05fin4/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -30 gpurun_out/r05fin4/gpu.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05fin4/checks.log 2>&1
rc=$?; tail -n1 gpurun_out/r05fin4/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05fin4/checks.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05fin4/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r05fin4/smoke.log; exit 1; }
tail -n1 gpurun_out/r05fin4/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05fin4/bench_driver.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r05fin4/bench_driver.log; exit 1; }
tail -n1 gpurun_out/r05fin4/bench_driver.log | cut -c1-300
timeout -k 10 900 bash tools/prof_headline.sh r05rtt2 rtt > gpurun_out/r05fin4/prof.log 2>&1 || { echo PROF FAIL; tail -20 gpurun_out/r05fin4/prof.log; exit 1; }
tail -n5 gpurun_out/r05fin4/prof.log
