#!/bin/bash
# Round 6, step X: the shipped libraries (rebuilt after the last source
# change) on the GPU: the GPU suite, the checks build's parity tests, smoke,
# the driver's command.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r06x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1
rc=$?; tail -n1 $O/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -40 $O/gpu.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py tests/test_host_components.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/checks.log 2>&1
rc=$?; tail -n1 $O/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 $O/checks.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 $O/smoke.log; exit 1; }
tail -n1 $O/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo BENCH FAIL; tail -20 $O/bench.log; exit 1; }
tail -n1 $O/bench.log | cut -c1-200
