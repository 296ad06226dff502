#!/bin/bash
# Round 5: shared-list placement tests (prod + checks), Pacman phase stamps.
set -o pipefail
mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 200 --timeout-method thread -k "shared_list or headline_config_4096 or golden" > gpurun_out/r05h/prod.log 2>&1
rc=$?; tail -2 gpurun_out/r05h/prod.log; [ $rc -eq 0 ] || { echo "PROD rc=$rc"; tail -40 gpurun_out/r05h/prod.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests/test_engine_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread -k "shared_list" > gpurun_out/r05h/checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05h/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -40 gpurun_out/r05h/checks.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps_pac.py > gpurun_out/r05h/stamps_pac.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r05h/stamps_pac.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05h/stamps_pac.log
