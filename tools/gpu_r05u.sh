#!/bin/bash
# Round 5: work-ordered dispatch of one-wave rollouts (GW_ORDERED=1): parity
# (rollouts vs steps, the timed launch shape vs the oracle, shards), A/B on the
# driver's command, tail probe.
set -o pipefail
mkdir -p gpurun_out/r05u
export TMPDIR=/tmp
GW_ORDERED=1 timeout -k 10 900 python -u -m pytest tests/test_rollout.py tests/test_engine_oracle.py tests/test_shard_engine.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rollout or timed_launch or shard" > gpurun_out/r05u/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05u/tests.log; [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; tail -30 gpurun_out/r05u/tests.log; exit 1; }
timeout -k 10 900 bash tools/ab_env.sh r05u/ab_ordered "off=- on=GW_ORDERED=1" || exit 1
timeout -k 10 900 bash tools/ab_env.sh r05u/ab_ordered_f100 "off=- on=GW_ORDERED=1" --steps 300 --warmup 5 || exit 1
GW_ORDERED=1 GW_ENGINE_VARIANT=stamps timeout -k 10 200 python3 tools/tail_probe.py --reps 2 > gpurun_out/r05u/tail_on.log 2>&1 || { echo "tail probe failed"; tail -5 gpurun_out/r05u/tail_on.log; exit 1; }
grep -E 'launch span|SIMDs by envs|per-SIMD last end' gpurun_out/r05u/tail_on.log
