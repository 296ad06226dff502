#!/bin/bash
# round-3 session f: Pacman turn rollout, cost of the observation stores
set -o pipefail
B=abmarl_amd/_build
: > gpurun_out/ab_f.jsonl
for L in libgw_engine.so libgw_engine_pacobs.so libgw_engine_pacnost.so libgw_engine_pacaux0.so libgw_engine_pacobs.so libgw_engine_pacnost.so libgw_engine_pacaux0.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --workload pacman --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/f_pac.log 2>&1 || { tail -20 gpurun_out/f_pac.log; exit 1; }
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/f_pac.log)}" >> gpurun_out/ab_f.jsonl
done
