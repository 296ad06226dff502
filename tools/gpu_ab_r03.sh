#!/bin/bash
# round-3 A/B + parity + profile session (one gpurun call)
set -o pipefail
B=abmarl_amd/_build
timeout -k 10 300 python3 tools/ab_headline.py $B/libgw_engine.so $B/libgw_engine_fp0.so $B/libgw_engine.so $B/libgw_engine_fp0.so \
    > gpurun_out/ab_head.jsonl 2> gpurun_out/ab_head.err || exit 1
timeout -k 10 300 python3 tools/ab_maze.py $B/libgw_engine.so $B/libgw_engine_fp0.so $B/libgw_engine_pd8.so $B/libgw_engine.so \
    > gpurun_out/ab_maze.jsonl 2> gpurun_out/ab_maze.err || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_engine_oracle.py tests/test_rollout.py tests/test_lane_kernel.py tests/test_pacman_engine.py tests/test_engine_golden.py \
    > gpurun_out/tests_sub.log 2>&1 || exit 1
bash tools/prof_headline.sh r03d || exit 1
bash tools/strong_proxy.sh
