#!/bin/bash
# Round 5: config 4's crowded draws -- the serial form (wave 0) below a pair
# count threshold: parity on the threshold-64 build, then the A/B.
set -o pipefail
mkdir -p gpurun_out/r05s
export TMPDIR=/tmp
GW_ENGINE_LIB=abmarl_amd/_build/ab/par64/libgw_engine.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "reach_the_target or rtt or workgroup" > gpurun_out/r05s/par64_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05s/par64_tests.log; [ $rc -eq 0 ] || { echo "PAR64 rc=$rc"; tail -30 gpurun_out/r05s/par64_tests.log; exit 1; }
A=abmarl_amd/_build/ab
timeout -k 10 900 bash tools/ab_libs.sh r05s/ab_rtt "head=- p16=$A/par16/libgw_engine.so p32=$A/par32/libgw_engine.so p64=$A/par64/libgw_engine.so" --workload rtt --steps 100 --warmup 5 || exit 1
