#!/bin/bash
# A/B of engine builds on the driver's headline command, alternating, 3 rounds.
#   bash tools/ab_libs.sh OUT "name=lib ..." [bench args]
# lib "-" = the main build.  -> gpurun_out/OUT.jsonl
set -o pipefail
OUT=$1; ARMS=$2; shift 2
ARGS=${*:-"--steps 20 --warmup 5"}
mkdir -p gpurun_out
: > gpurun_out/$OUT.jsonl
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in $ARMS; do
    name=${arm%%=*}; lib=${arm#*=}
    if [ "$lib" = "-" ]; then unset GW_ENGINE_LIB; else export GW_ENGINE_LIB=$lib; fi
    timeout -k 10 120 python3 bench.py $ARGS --no-other --no-cpu-baseline \
        > gpurun_out/${OUT}_run.log 2>&1 || { echo "bench $name failed"; tail -5 gpurun_out/${OUT}_run.log; exit 1; }
    python3 -c "
import json
d = json.loads(open('gpurun_out/${OUT}_run.log').read().strip().splitlines()[-1])
print(json.dumps({'arm': '$name', 'round': $r, 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/$OUT.jsonl
  done
done
unset GW_ENGINE_LIB
cat gpurun_out/$OUT.jsonl
