#!/bin/bash
# Round 5 HEAD: the whole GPU suite, smoke, the headline rocprof/PMC evidence,
# the driver's default bench line.
set -o pipefail
mkdir -p gpurun_out/r05p
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p/gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05p/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 gpurun_out/r05p/gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05p/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r05p/smoke.log; exit 1; }
tail -2 gpurun_out/r05p/smoke.log
timeout -k 10 600 bash tools/prof_headline.sh r05 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r05p/bench_default.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r05p/bench_default.log; exit 1; }
tail -1 gpurun_out/r05p/bench_default.log
