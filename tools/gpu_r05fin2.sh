#!/bin/bash
# Round 5 HEAD (reset weight 384): the whole GPU suite, smoke, the driver's command.
set -o pipefail
mkdir -p gpurun_out/r05fin2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05fin2/gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05fin2/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 gpurun_out/r05fin2/gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05fin2/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r05fin2/smoke.log; exit 1; }
tail -1 gpurun_out/r05fin2/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05fin2/bench_driver.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r05fin2/bench_driver.log; exit 1; }
tail -1 gpurun_out/r05fin2/bench_driver.log | cut -c1-600
