#!/bin/bash
# round-3 session n: remaining-work issue priority (GW_PROGRESS_PRIO=2) vs progress priority
set -o pipefail
B=abmarl_amd/_build
timeout -k 10 500 python3 tools/ab_headline.py $B/libgw_engine.so $B/libgw_engine_prw.so $B/libgw_engine_prw2.so \
    $B/libgw_engine.so $B/libgw_engine_prw.so $B/libgw_engine_prw2.so > gpurun_out/ab_head_n.jsonl 2> gpurun_out/ab_head_n.err || exit 1
: > gpurun_out/ab_n_s20.jsonl
for L in libgw_engine.so libgw_engine_prw.so libgw_engine.so libgw_engine_prw.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/n_s20.log 2>&1 || exit 1
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/n_s20.log)}" >> gpurun_out/ab_n_s20.jsonl
done
