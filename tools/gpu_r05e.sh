#!/bin/bash
# Round 5 measurements on HEAD: env-map A/B + tail probe, config 4 and
# headline rocprof/PMC evidence, Pacman SQ/PMC, the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 bash tools/ab_swz.sh "0 -1 16" || exit 1
timeout -k 10 400 bash tools/prof_headline.sh r05rtt rtt || exit 1
timeout -k 10 400 bash tools/pmc_pacman.sh r05 || exit 1
