#!/bin/bash
# Round 6, step Z: config 4 per-phase stamps on the shipped stamps build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python3 tools/stamps.py rtt 1024 > $O/stamps_rtt.log 2>&1 || { echo STAMPS FAIL; tail -20 $O/stamps_rtt.log; exit 1; }
grep -A30 "rtt: step launch" $O/stamps_rtt.log | head -32
