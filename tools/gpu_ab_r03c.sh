#!/bin/bash
# round-3 session c: lane-group maze kernel variant (rollout-protocol
# instantiation, branch-free move / observation) -- parity, then A/B
set -o pipefail
B=abmarl_amd/_build
GW_ENGINE_LIB=$B/libgw_engine_lanebf.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_lane_kernel.py tests/test_maze_engine.py tests/test_rollout.py tests/test_engine_oracle.py \
    > gpurun_out/tests_c.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_maze.py $B/libgw_engine.so $B/libgw_engine_lanebf.so $B/libgw_engine.so $B/libgw_engine_lanebf.so \
    > gpurun_out/ab_maze_c.jsonl 2> gpurun_out/ab_maze_c.err
