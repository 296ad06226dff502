#!/bin/bash
# rocprofv3 evidence for one bench workload, on the GPU box:
#   tools/profile.sh <tag> [team_battle|rtt|maze] [rollout|step] [fragment]
# 1. --kernel-trace --stats over a bench run (per-kernel durations);
# 2. two separate --pmc passes, FETCH_SIZE and WRITE_SIZE (they do not fit
#    one pass on gfx950), over a short run of the same workload.
# rollout mode: every step_kernel dispatch is a gw_rollout fragment of
# <fragment> steps (default 100; 20 is the driver's `--steps 20` run), the
# pre-roll, warmup and timed steps alike.
# Raw outputs go under gpurun_out/prof_<tag>_*; tools/summarize_profile.py
# turns them into profiles/<tag>_*.
set -o pipefail
TAG=${1:?tag}
WL=${2:-team_battle}
MODE=${3:-rollout}
FRAG=${4:-100}
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
BENCH="$ROOT/bench.py --workload $WL --mode $MODE --no-cpu-baseline --no-other --fragment $FRAG"
if [ "$MODE" = rollout ]; then
  STATS_ARGS="--steps 200 --warmup 100 --preroll 900"; PMC_ARGS="--steps $FRAG --warmup 0 --preroll 100"
else
  STATS_ARGS="--steps 200 --warmup 20"; PMC_ARGS="--steps 30 --warmup 5"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_stats" -o run \
    -- python3 $BENCH $STATS_ARGS > "$OUT/prof_${TAG}_stats.log" 2>&1 \
    || { echo "stats pass failed"; tail -20 "$OUT/prof_${TAG}_stats.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/prof_${TAG}_$C" -o run \
        -- python3 $BENCH $PMC_ARGS > "$OUT/prof_${TAG}_$C.log" 2>&1 \
        || { echo "$C pass failed"; tail -20 "$OUT/prof_${TAG}_$C.log"; exit 1; }
done
python3 "$ROOT/tools/summarize_profile.py" "$TAG" "$WL" --mode "$MODE" --raw "$OUT" --dest "$OUT/profiles_$TAG" \
    --stats-args "$STATS_ARGS" --pmc-args "$PMC_ARGS" --fragment "$FRAG"
