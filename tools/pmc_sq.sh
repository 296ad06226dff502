#!/bin/bash
# SQ instruction / cycle counters of the step kernel (separate --pmc passes,
# kernel-trace only; MI355X_MICROARCH.md profiling rules).
#   bash tools/pmc_sq.sh <tag>   -> gpurun_out/pmc_<tag>/
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline --no-other --steps 30 --warmup 5"
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "PMC pass $i FAIL"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'step_kernel' in r['Kernel_Name']:
            vals[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(f"{k:24s} mean/launch {sum(v)/len(v):14.1f}  (n={len(v)})")
PY
