#!/bin/bash
# round-3 session m: the headline kernel without the action prefetch -- parity, A/B
set -o pipefail
B=abmarl_amd/_build
GW_ENGINE_LIB=$B/libgw_engine_pref0.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_engine_oracle.py tests/test_rollout.py tests/test_engine_golden.py tests/test_dict_api.py \
    > gpurun_out/tests_m.log 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_headline.py $B/libgw_engine.so $B/libgw_engine_pref0.so $B/libgw_engine.so $B/libgw_engine_pref0.so \
    $B/libgw_engine.so $B/libgw_engine_pref0.so > gpurun_out/ab_head_m.jsonl 2> gpurun_out/ab_head_m.err
