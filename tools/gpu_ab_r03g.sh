#!/bin/bash
# round-3 session g: Pacman observation as dwordx4 quads, crowded list by (row, col)
set -o pipefail
B=abmarl_amd/_build
GW_ENGINE_LIB=$B/libgw_engine_pacq.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pacman_engine.py tests/test_components_f3.py tests/test_rollout.py tests/test_dict_api.py \
    > gpurun_out/tests_g.log 2>&1 || exit 1
: > gpurun_out/ab_g.jsonl
for L in libgw_engine.so libgw_engine_pacq.so libgw_engine.so libgw_engine_pacq.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --workload pacman --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/g_pac.log 2>&1 || { tail -20 gpurun_out/g_pac.log; exit 1; }
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/g_pac.log)}" >> gpurun_out/ab_g.jsonl
done
