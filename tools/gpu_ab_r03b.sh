#!/bin/bash
# round-3 session b: parity of the Pacman / workgroup-kernel changes, then
# A/B of HEAD's library against the round-start one (fp0) on configs 5 and 4
set -o pipefail
B=abmarl_amd/_build
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pacman_engine.py tests/test_components_f3.py tests/test_rollout.py tests/test_engine_oracle.py \
    tests/test_engine_golden.py tests/test_components.py > gpurun_out/tests_b.log 2>&1 || exit 1
: > gpurun_out/ab_b.jsonl
for W in pacman rtt; do
  for L in libgw_engine.so libgw_engine_fp0.so libgw_engine.so libgw_engine_fp0.so; do
    GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --workload $W --steps 200 --warmup 5 --no-other --no-cpu-baseline \
        > gpurun_out/b_${W}.log 2>&1 || { tail -20 gpurun_out/b_${W}.log; exit 1; }
    echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/b_${W}.log)}" >> gpurun_out/ab_b.jsonl
  done
done
