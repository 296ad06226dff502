#!/bin/bash
# SQ / HBM counters of pac_kernel on BASELINE config 5 (Pacman, 16384 envs,
# TurnBasedManager): bench.py --workload pacman, one --pmc pass per counter
# set (kernel-trace only; MI355X_MICROARCH.md's per-block limits), summed
# per pac_kernel dispatch of the timed turn rollouts.
#   bash tools/pmc_pacman.sh <tag>   -> gpurun_out/pmc_pac_<tag>/, summary.txt
set -o pipefail
TAG=${1:-pac}
OUT=gpurun_out/pmc_pac_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --workload pacman --steps 100 --warmup 5 --preroll 200 --no-cpu-baseline --no-other"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD \
    > $OUT/stats.log 2>&1 || { echo "stats pass failed"; tail -20 $OUT/stats.log; exit 1; }
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- $CMD \
      > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($SET) failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" > $OUT/summary.txt <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'pac_kernel' in r['Kernel_Name']:
            key = (r['Kernel_Name'].split('(')[0][-40:], r.get('Dispatch_Id', r.get('Correlation_Id', '?')))
            vals[key][r['Counter_Name']] += float(r['Counter_Value'])
per = collections.defaultdict(list)
for (kn, _), d in vals.items():
    for c, v in d.items():
        per[(kn, c)].append(v)
for (kn, c), v in sorted(per.items()):
    print(f"{kn:42s} {c:22s} mean/dispatch {sum(v)/len(v):16.1f}  n={len(v)}")
for f in glob.glob(out + '/stats/**/*kernel_stats.csv', recursive=True):
    print(open(f).read())
PY
cat $OUT/summary.txt | head -60
