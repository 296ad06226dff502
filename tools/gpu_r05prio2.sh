#!/bin/bash
# Round 5: GW_PRIO_RESET_W 192 (HEAD) vs 384 vs 768, 8 alternating rounds of
# the driver's command, then 100-step fragments.
set -o pipefail
mkdir -p gpurun_out/r05prio
export TMPDIR=/tmp
A=abmarl_amd/_build/ab
ROUNDS=8 timeout -k 10 1000 bash tools/ab_libs.sh r05prio/ab_prio8 "w192=- w384=$A/prio384/libgw_engine.so w768=$A/prio768/libgw_engine.so" || exit 1
ROUNDS=4 timeout -k 10 1000 bash tools/ab_libs.sh r05prio/ab_prio_f100 "w192=- w384=$A/prio384/libgw_engine.so w768=$A/prio768/libgw_engine.so" --steps 300 --warmup 5 || exit 1
