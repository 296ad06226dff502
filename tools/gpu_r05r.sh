#!/bin/bash
# Round 5: Pacman with the baked-in action prefetch (parity); config 4's
# crowded-draw sub-phases (stamps); Pacman phase stamps.
set -o pipefail
mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pacman_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05r/pac_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05r/pac_tests.log; [ $rc -eq 0 ] || { echo "PAC rc=$rc"; tail -30 gpurun_out/r05r/pac_tests.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r05r/stamps_rtt.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r05r/stamps_rtt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05r/stamps_rtt.log | tail -25
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps_pac.py > gpurun_out/r05r/stamps_pac.log 2>&1 || { echo STAMPS PAC FAIL; tail -20 gpurun_out/r05r/stamps_pac.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05r/stamps_pac.log
