#!/bin/bash
# Round 5: config 4's crowded-cell offset passes on wave 0 alone (DPP scans,
# no workgroup barrier per pass) when the pairs fit one wave -- the GPU suite,
# checks build, stamps (new vs GW_CROWD_ONE_WAVE=0), A/B of the rtt bench.
set -o pipefail
mkdir -p gpurun_out/r05cw
export TMPDIR=/tmp
A=abmarl_amd/_build/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05cw/gpu.log 2>&1
rc=$?; tail -n1 gpurun_out/r05cw/gpu.log; [ $rc -eq 0 ] || { echo "GPU rc=$rc"; tail -30 gpurun_out/r05cw/gpu.log; exit 1; }
GW_ENGINE_VARIANT=checks timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05cw/checks.log 2>&1
rc=$?; tail -n1 gpurun_out/r05cw/checks.log; [ $rc -eq 0 ] || { echo "CHECKS rc=$rc"; tail -30 gpurun_out/r05cw/checks.log; exit 1; }
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r05cw/stamps_rtt.log 2>&1 || { echo STAMPS FAIL; exit 1; }
GW_ENGINE_VARIANT=stamps GW_ENGINE_LIB=$A/scw0/libgw_engine.so timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r05cw/stamps_rtt_cw0.log 2>&1 || { echo STAMPS0 FAIL; exit 1; }
echo new; grep -E 'crowd|pairs|step launch|whole' gpurun_out/r05cw/stamps_rtt.log
echo cw0; grep -E 'crowd|pairs|whole' gpurun_out/r05cw/stamps_rtt_cw0.log
ROUNDS=4 timeout -k 10 900 bash tools/ab_libs.sh r05cw/ab_rtt "cw0=$A/cw0/libgw_engine.so new=-" --workload rtt --steps 100 --warmup 5 || exit 1
