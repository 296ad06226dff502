#!/bin/bash
# Round 5: the Jacobi placement ends without a confirming sweep when no moved
# estimate can change a fixpoint -- parity (prod + checks), stamps (new vs
# GW_JAC_CONFIRM=0), A/B on the driver's command and the closed loop.
set -o pipefail
mkdir -p gpurun_out/r05conf
export TMPDIR=/tmp
A=abmarl_amd/_build/ab
timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py tests/test_components.py tests/test_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05conf/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05conf/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05conf/tests.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05conf/checks.log 2>&1
rc=$?; tail -1 gpurun_out/r05conf/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05conf/checks.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r05conf/stamps_tb.log 2>&1 || { echo STAMPS FAIL; exit 1; }
GW_ENGINE_VARIANT=stamps GW_ENGINE_LIB=$A/stc0/libgw_engine.so timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r05conf/stamps_tb_conf0.log 2>&1 || { echo STAMPS0 FAIL; exit 1; }
echo new; grep -E 'placement|jacobi' gpurun_out/r05conf/stamps_tb.log
echo conf0; grep -E 'placement|jacobi' gpurun_out/r05conf/stamps_tb_conf0.log
ROUNDS=6 timeout -k 10 900 bash tools/ab_libs.sh r05conf/ab_headline "conf0=$A/conf0/libgw_engine.so new=-" || exit 1
timeout -k 10 900 bash tools/ab_libs.sh r05conf/ab_closed "conf0=$A/conf0/libgw_engine.so new=-" --mode step --steps 300 --warmup 20 || exit 1
