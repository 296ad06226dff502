#!/bin/bash
# Strong-scaling proxy on one GPU: the headline workload at the
# per-rank env counts of a 4096-GLOBAL-env job on 8/4/2/1 GPUs, 100-step
# fragments, 200 timed steps -> gpurun_out/strong_proxy.jsonl; then the
# small-batch counts (512, 1024) on the workgroup kernel with 1, 2 and 4
# waves per env (bench.py --workgroup-waves) -> gpurun_out/strong_proxy_wg.jsonl
set -o pipefail
OUT=gpurun_out/strong_proxy.jsonl
: > $OUT
for E in 512 1024 2048 4096; do
  timeout -k 10 180 python3 bench.py --envs $E --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/sp_$E.log 2>&1 || { echo "envs $E failed"; tail -20 gpurun_out/sp_$E.log; exit 1; }
  grep '^{' gpurun_out/sp_$E.log >> $OUT
done
OUT=gpurun_out/strong_proxy_wg.jsonl
: > $OUT
for W in 1 2 4; do
  for E in 512 1024; do
    timeout -k 10 180 python3 bench.py --envs $E --steps 200 --warmup 5 --no-other --no-cpu-baseline \
        --workgroup-waves $W > gpurun_out/spw_${W}_$E.log 2>&1 || { echo "waves $W envs $E failed"; tail -20 gpurun_out/spw_${W}_$E.log; exit 1; }
    grep '^{' gpurun_out/spw_${W}_$E.log >> $OUT
  done
done
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open('gpurun_out/strong_proxy.jsonl')]
full = [r for r in rows if r['config']['envs_per_gpu'] == 4096][0]['value']
for f in ('gpurun_out/strong_proxy.jsonl', 'gpurun_out/strong_proxy_wg.jsonl'):
    for r in map(json.loads, open(f)):
        print(f"{r['config']['workload'][:90]:90s} envs {r['config']['envs_per_gpu']:5d} value {r['value']:.4g} "
              f"launch {r['roofline']['kernel_ms']:.3f} ms  proxy {r['value'] / full:.3f}")
PY
