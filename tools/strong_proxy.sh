#!/bin/bash
# Strong-scaling proxy on one GPU: the headline workload at the
# per-rank env counts of a 4096-GLOBAL-env job on 8/4/2/1 GPUs, 100-step
# fragments, 200 timed steps -> gpurun_out/strong_proxy.jsonl
set -o pipefail
OUT=gpurun_out/strong_proxy.jsonl
: > $OUT
for E in 512 1024 2048 4096; do
  timeout -k 10 180 python3 bench.py --envs $E --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/sp_$E.log 2>&1 || { echo "envs $E failed"; tail -20 gpurun_out/sp_$E.log; exit 1; }
  grep '^{' gpurun_out/sp_$E.log >> $OUT
done
