#!/bin/bash
# Round 5: config 4 one-wave crowded draws, second step: wave 0 also ranks the
# members and buffers the words (three workgroup barriers fewer) -- the GPU
# suite, checks build, stamps and the rtt bench vs the first step (c1).
set -o pipefail
mkdir -p gpurun_out/r05cw2
export TMPDIR=/tmp
A=abmarl_amd/_build/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05cw2/gpu.log 2>&1
rc=$?; tail -n1 gpurun_out/r05cw2/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -30 gpurun_out/r05cw2/gpu.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05cw2/checks.log 2>&1
rc=$?; tail -n1 gpurun_out/r05cw2/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05cw2/checks.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r05cw2/stamps_rtt.log 2>&1 || { echo STAMPS FAIL; exit 1; }
GW_ENGINE_VARIANT=stamps GW_ENGINE_LIB=$A/sc1/libgw_engine.so timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r05cw2/stamps_rtt_c1.log 2>&1 || { echo STAMPS0 FAIL; exit 1; }
echo new; grep -E 'crowd|pairs|step launch|whole' gpurun_out/r05cw2/stamps_rtt.log
echo c1; grep -E 'crowd|pairs|whole' gpurun_out/r05cw2/stamps_rtt_c1.log
ROUNDS=4 timeout -k 10 900 bash tools/ab_libs.sh r05cw2/ab_rtt "c1=$A/c1/libgw_engine.so new=-" --workload rtt --steps 100 --warmup 5 || exit 1
