#!/bin/bash
# A/B of an environment setting on the driver's headline command, alternating,
# 3 rounds:  bash tools/ab_env.sh OUT "name=VAR=value ..." [bench args]
# ("name=-" runs without any setting) -> gpurun_out/OUT.jsonl
set -o pipefail
OUT=$1; ARMS=$2; shift 2
ARGS=${*:-"--steps 20 --warmup 5"}
mkdir -p gpurun_out/$(dirname $OUT)
: > gpurun_out/$OUT.jsonl
for r in 1 2 3; do
  for arm in $ARMS; do
    name=${arm%%=*}; kv=${arm#*=}
    if [ "$kv" = "-" ]; then envs=""; else envs="$kv"; fi
    env $envs timeout -k 10 120 python3 bench.py $ARGS --no-other --no-cpu-baseline \
        > gpurun_out/${OUT}_run.log 2>&1 || { echo "bench $name failed"; tail -5 gpurun_out/${OUT}_run.log; exit 1; }
    python3 -c "
import json
d = json.loads(open('gpurun_out/${OUT}_run.log').read().strip().splitlines()[-1])
print(json.dumps({'arm': '$name', 'round': $r, 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/$OUT.jsonl
  done
done
cat gpurun_out/$OUT.jsonl
