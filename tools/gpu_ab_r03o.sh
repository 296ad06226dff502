#!/bin/bash
# round-3 session o: remaining-work priority, reset weight 192 vs 400, the driver's command
set -o pipefail
B=abmarl_amd/_build
: > gpurun_out/ab_o_s20.jsonl
for L in libgw_engine.so libgw_engine_prw.so libgw_engine_prw2.so libgw_engine.so libgw_engine_prw.so libgw_engine_prw2.so libgw_engine.so libgw_engine_prw.so libgw_engine_prw2.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/o_s20.log 2>&1 || exit 1
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/o_s20.log)}" >> gpurun_out/ab_o_s20.jsonl
done
GW_ENGINE_LIB=$B/libgw_engine_prw2.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_engine_oracle.py tests/test_rollout.py > gpurun_out/tests_o.log 2>&1
