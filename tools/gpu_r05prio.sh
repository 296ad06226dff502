#!/bin/bash
# Round 5: the pending-reset weight of the remaining-work issue priority
# (GW_PRIO_RESET_W, 192 in HEAD) re-tuned on the driver's command.
set -o pipefail
mkdir -p gpurun_out/r05prio
export TMPDIR=/tmp
A=abmarl_amd/_build/ab
timeout -k 10 1000 bash tools/ab_libs.sh r05prio/ab_prio "w192=- w0=$A/prio0/libgw_engine.so w384=$A/prio384/libgw_engine.so w768=$A/prio768/libgw_engine.so" || exit 1
