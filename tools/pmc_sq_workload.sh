#!/bin/bash
# SQ instruction / cycle counters of one workload's step kernel over a short
# bench run (one --pmc pass per set, kernel trace only):
#   bash tools/pmc_sq_workload.sh <tag> <maze|pacman|team_battle|rtt> [bench args]
#   -> gpurun_out/sq_<tag>/ and a per-dispatch table on stdout
set -o pipefail
TAG=${1:?tag}
WL=${2:?workload}
shift 2
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --workload $WL --no-other --no-cpu-baseline --steps 20 --warmup 5 --preroll 200 $*"
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 \
      || { echo "PMC pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" "$WL" <<'PY'
import csv, glob, sys, collections
out, wl = sys.argv[1], sys.argv[2]
k = {'maze': 'lane_step_kernel', 'pacman': 'pac_kernel', 'team_battle': 'step_kernel', 'rtt': 'wg_step_kernel'}[wl]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name']
        if k in name and 'random' not in name and (k != 'step_kernel' or 'lane_' not in name and 'wg_' not in name):
            vals[r['Counter_Name']][int(r['Dispatch_Id'])] += float(r['Counter_Value'])
for c, d in sorted(vals.items()):
    v = [d[x] for x in sorted(d)]
    print(f"{c:24s} last dispatch {v[-1]:14.0f}   mean {sum(v)/len(v):14.0f}  (n={len(v)})")
PY
