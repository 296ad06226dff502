#!/bin/bash
# rocprofv3 evidence for the headline line, on the GPU box, at the driver's
# own workload (bench.py --gpus 1 --steps 20 --warmup 5: 1000-step pre-roll,
# ONE timed 20-step gw_rollout launch):
#   bash tools/prof_headline.sh <tag> [rtt]   -> gpurun_out/ph_<tag>/
# (rtt: BASELINE config 4's line, bench.py --workload rtt --steps 100 --warmup 5;
#  pacman: config 5's turn rollout, --workload pacman --steps 50 --warmup 5,
#  ONE timed 50-turn gw_turn_rollout launch)
# 1. --kernel-trace --stats over the driver's exact command;
# 2. FETCH_SIZE and WRITE_SIZE, one --pmc pass each, same workload with the
#    other configs and the CPU baseline skipped (--no-other --no-cpu-baseline:
#    the headline run itself is unchanged);
# 3. three SQ counter passes (instruction mix, wait/busy cycles, LDS bank
#    conflicts) on the same workload.
# tools/summarize_headline.py turns them into profiles/<tag>_* and
# profiles/pmc_step_kernel_rollout_f20.json.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/ph_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
WL=${2:-team_battle}
if [ "$WL" = rtt ]; then
  CMD="python3 bench.py --gpus 1 --workload rtt --steps 100 --warmup 5"
elif [ "$WL" = pacman ]; then
  CMD="python3 bench.py --gpus 1 --workload pacman --steps 50 --warmup 5"
else
  CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD \
    > $OUT/stats.log 2>&1 || { echo "stats pass failed"; tail -20 $OUT/stats.log; exit 1; }
SHORT="$CMD --no-other --no-cpu-baseline"
i=0
for SET in FETCH_SIZE WRITE_SIZE \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- $SHORT \
      > $OUT/p$i.log 2>&1 || { echo "PMC pass $i ($SET) failed"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 tools/summarize_headline.py $TAG --raw $OUT --dest $OUT/profiles --workload $WL
