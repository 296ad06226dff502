#!/bin/bash
# round-3 session k: the written rows stored as row-aligned dwordx4 chunks
# (GW_OBS_ROW_STORE) -- parity on the variant, then A/B
set -o pipefail
B=abmarl_amd/_build
GW_ENGINE_LIB=$B/libgw_engine_rowst.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_engine_oracle.py tests/test_rollout.py tests/test_engine_golden.py tests/test_dict_api.py tests/test_components.py \
    > gpurun_out/tests_k.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_headline.py $B/libgw_engine.so $B/libgw_engine_rowst.so $B/libgw_engine.so $B/libgw_engine_rowst.so \
    > gpurun_out/ab_head_k.jsonl 2> gpurun_out/ab_head_k.err
