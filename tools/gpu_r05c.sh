#!/bin/bash
# Round 5: HEAD (MT key LDS-typed everywhere, observe_big inlined: no scratch in
# the generic-window kernels) in FRESH processes that start with
# rtt_16_example's reset_kernel<0> -- the order in which 95ec8c4's probe2
# variant faulted at its first reset -- then the checks selection and the
# production GPU suite.
set -o pipefail
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
GW_ENGINE_VARIANT=checks timeout -k 10 120 python -u tools/fault_r05/probe.py rtt_16_example rtt_16 > gpurun_out/r05c/head_checks_fresh.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05c/head_checks_fresh.log | cut -c1-400; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/fault_r05/probe.py rtt_16_example rtt_16 > gpurun_out/r05c/head_prod_fresh.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05c/head_prod_fresh.log | cut -c1-400; [ $rc -eq 0 ] || exit 1
SEL="oracle or golden or rollout or components or shard or builders or kernel_resources"
GW_ENGINE_VARIANT=checks timeout -k 10 700 python -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "$SEL" > gpurun_out/r05c/head_checks.log 2>&1
rc=$?; tail -2 gpurun_out/r05c/head_checks.log; [ $rc -eq 0 ] || { echo "HEAD CHECKS rc=$rc"; tail -40 gpurun_out/r05c/head_checks.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c/head_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r05c/head_gpu.log; [ $rc -eq 0 ] || { echo "HEAD GPU rc=$rc"; tail -40 gpurun_out/r05c/head_gpu.log; exit 1; }
# headline tail: per-SIMD placement of the envs that reach the horizon in the fragment
GW_ENGINE_VARIANT=stamps timeout -k 10 200 python -u tools/tail_probe.py --reps 2 > gpurun_out/r05c/tail_probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r05c/tail_probe.log | head -60; [ $rc -eq 0 ] || exit 1
