#!/bin/bash
# round-3 session e: Pacman full-grid observation fast path -- parity, A/B
set -o pipefail
B=abmarl_amd/_build
GW_ENGINE_LIB=$B/libgw_engine_pacpre.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pacman_engine.py tests/test_components_f3.py tests/test_rollout.py tests/test_dict_api.py \
    > gpurun_out/tests_e.log 2>&1 || exit 1
: > gpurun_out/ab_e.jsonl
for L in libgw_engine.so libgw_engine_pacpre.so libgw_engine.so libgw_engine_pacpre.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --workload pacman --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/e_pac.log 2>&1 || { tail -20 gpurun_out/e_pac.log; exit 1; }
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/e_pac.log)}" >> gpurun_out/ab_e.jsonl
done
