#!/bin/bash
# round-3 session l: the headline kernel's tuning switches re-checked on HEAD
set -o pipefail
B=abmarl_amd/_build
timeout -k 10 500 python3 tools/ab_headline.py $B/libgw_engine.so $B/libgw_engine_prio0.so $B/libgw_engine_pref0.so $B/libgw_engine_aux0h.so \
    $B/libgw_engine.so $B/libgw_engine_prio0.so $B/libgw_engine_pref0.so $B/libgw_engine_aux0h.so > gpurun_out/ab_head_l.jsonl 2> gpurun_out/ab_head_l.err
