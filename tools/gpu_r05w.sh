#!/bin/bash
# Round 5: placement sweeps skip the list lengths and draws when no fresh set
# changed -- parity (prod + checks), A/B on the driver's command, stamps.
set -o pipefail
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py tests/test_components.py tests/test_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05w/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05w/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05w/tests.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05w/checks.log 2>&1
rc=$?; tail -1 gpurun_out/r05w/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05w/checks.log; exit 1; }
timeout -k 10 900 bash tools/ab_libs.sh r05w/ab_headline "base=abmarl_amd/_build/ab/h2/libgw_engine.so new=-" || exit 1
timeout -k 10 900 bash tools/ab_libs.sh r05w/ab_closed "base=abmarl_amd/_build/ab/h2/libgw_engine.so new=-" --mode step --steps 300 --warmup 20 || exit 1
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r05w/stamps_tb.log 2>&1 || { echo STAMPS FAIL; exit 1; }
grep -E 'placement|jacobi' gpurun_out/r05w/stamps_tb.log
