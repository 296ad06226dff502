#!/bin/bash
# PC sampling (rocprofv3 host_trap, beta) over a short TeamBattle rollout:
# where the step kernel's waves are, instruction by instruction.
#   bash tools/pcsample.sh <tag> [method] [interval]  -> gpurun_out/pcs_<tag>/
set -o pipefail
TAG=${1:-pcs}
METHOD=${2:-host_trap}
INTERVAL=${3:-1}
OUT=gpurun_out/pcs_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD \
    --pc-sampling-unit time --pc-sampling-interval $INTERVAL --output-format csv -d $OUT -o run \
    -- python3 tools/rollout_run.py --frags 3 --skip > $OUT.log 2>&1
