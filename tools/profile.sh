#!/bin/bash
# rocprofv3 kernel trace + stats and separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# usage: bash tools/profile.sh <tag>   (writes gpurun_out/prof_<tag>/)
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --no-cpu-baseline --no-other"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH --steps 200 --warmup 20 > $OUT/trace.log 2>&1 || { echo TRACE FAIL; tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $BENCH --steps 30 --warmup 5 > $OUT/fetch.log 2>&1 || { echo FETCH FAIL; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $BENCH --steps 30 --warmup 5 > $OUT/write.log 2>&1 || { echo WRITE FAIL; tail -20 $OUT/write.log; exit 1; }
find $OUT -name '*.csv' | head -20
