#!/bin/bash
# Round 5 HEAD: pac_kernel SQ / HBM counters after the round's changes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 bash tools/pmc_pacman.sh r05final || exit 1
cat gpurun_out/pmc_pac_r05final/summary.txt | head -30
