#!/bin/bash
# round-3 closing run 3 (HEAD: remaining-work priority): GPU suite, smoke,
# the driver's command three times and with the reset weight 400 variant, default bench
set -o pipefail
B=abmarl_amd/_build
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
: > gpurun_out/ab_p_s20.jsonl
for L in libgw_engine.so libgw_engine_prw2.so libgw_engine.so libgw_engine_prw2.so libgw_engine.so libgw_engine_prw2.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/p_s20.log 2>&1 || exit 1
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/p_s20.log)}" >> gpurun_out/ab_p_s20.jsonl
done
timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py > gpurun_out/bench_final.log 2>&1
