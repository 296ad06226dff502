#!/bin/bash
# A/B of the one-wave step kernel's env map (block_env, GW_ENV_SWZ = Q) on the
# driver's headline command, alternating, 3 rounds; then the tail probe per Q.
# (Round 5; the knob was removed after the A/B, profiles/r05/ab_env_map/: the
# identity map stayed.)
#   bash tools/ab_swz.sh "0 4 16" -> gpurun_out/ab_swz.jsonl, gpurun_out/ab_swz_tail_<Q>.log
set -o pipefail
QS=${1:-"0 4 16"}
mkdir -p gpurun_out
: > gpurun_out/ab_swz.jsonl
for r in 1 2 3; do
  for q in $QS; do
    GW_ENV_SWZ=$q timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-other --no-cpu-baseline \
        > gpurun_out/ab_swz_run.log 2>&1 || { echo "bench Q=$q failed"; tail -5 gpurun_out/ab_swz_run.log; exit 1; }
    python3 -c "
import json,sys
d = json.loads(open('gpurun_out/ab_swz_run.log').read().strip().splitlines()[-1])
print(json.dumps({'Q': $q, 'round': $r, 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/ab_swz.jsonl
  done
done
cat gpurun_out/ab_swz.jsonl
for q in $QS; do
  GW_ENV_SWZ=$q GW_ENGINE_VARIANT=stamps timeout -k 10 200 python3 tools/tail_probe.py --reps 2 \
      > gpurun_out/ab_swz_tail_$q.log 2>&1 || { echo "tail probe Q=$q failed"; exit 1; }
  echo "== Q=$q"; grep -E 'launch span|SIMDs by envs|per-SIMD last end' gpurun_out/ab_swz_tail_$q.log
done
