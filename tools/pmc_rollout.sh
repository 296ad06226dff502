#!/bin/bash
# SQ counters of the fused rollout step kernel (tools/rollout_run.py), one
# --pmc pass per counter set, kernel trace only (MI355X_MICROARCH.md rules).
#   bash tools/pmc_rollout.sh <tag> [rollout_run.py args]   -> gpurun_out/pmc_<tag>/
set -o pipefail
TAG=${1:-roll}
shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- python3 tools/rollout_run.py --frags 2 "$@" > $OUT/p$i.log 2>&1 || { echo "PMC pass $i FAIL"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'step_kernel' in r['Kernel_Name'] and 'random' not in r['Kernel_Name']:
            vals[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(f"{k:24s} last two launches (the rollouts): " + ' '.join(f'{x:14.0f}' for x in v[-2:]) + f'   single-step mean {sum(v[:-2]) / max(1, len(v) - 2):12.0f}')
PY
