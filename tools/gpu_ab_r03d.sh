#!/bin/bash
# round-3 session d: Pacman turn rollout -- share of the observation (A/B
# against a build without it, timing only) and SQ counters of HEAD's kernel
set -o pipefail
B=abmarl_amd/_build
: > gpurun_out/ab_d.jsonl
for L in libgw_engine.so libgw_engine_pacnoobs.so libgw_engine.so libgw_engine_pacnoobs.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --workload pacman --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/d_pac.log 2>&1 || { tail -20 gpurun_out/d_pac.log; exit 1; }
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/d_pac.log)}" >> gpurun_out/ab_d.jsonl
done
bash tools/pmc_sq_workload.sh pac_r03 pacman > gpurun_out/sq_pac_r03.txt 2>&1
