#!/bin/bash
# A/B of engine library builds (tools/ab_lib.py) on one bench.py workload, on
# the GPU box: each library in its own fresh process, in the order given
#   bash tools/ab_bench.sh <team_battle|maze|rtt|pacman> <steps> <lib.so> [<lib.so> ...]
#   -> gpurun_out/ab_bench_<workload>[_<AB_TAG>].jsonl ({"lib": ..., "line": <bench JSON line>})
# (AB_ARGS: extra bench.py arguments, e.g. "--mode step")
set -o pipefail
W=${1:?workload}; N=${2:?steps}; shift 2
OUT=gpurun_out/ab_bench_$W${AB_TAG:+_$AB_TAG}.jsonl
: > $OUT
for L in "$@"; do
  GW_ENGINE_LIB=$L timeout -k 10 240 python3 bench.py --workload $W --steps $N --warmup 5 --no-other --no-cpu-baseline $AB_ARGS \
      > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/ab_bench.log)}" >> $OUT
done
