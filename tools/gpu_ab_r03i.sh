#!/bin/bash
# round-3 session i: (1) the workgroup kernel with one reset call site (wg2)
# and the out-of-line twist (tw, part 7): parity, A/B on configs 4 and the
# headline; (2) Pacman dwordx4 observation (pacq): parity, A/B; (3) the
# headline's observation store cost (nogst) and the written-rows store (cst)
set -o pipefail
B=abmarl_amd/_build
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
GW_ENGINE_LIB=$B/libgw_engine_tw.so timeout -k 10 600 $T tests/test_engine_oracle.py tests/test_engine_golden.py \
    tests/test_rollout.py tests/test_components.py tests/test_dict_api.py > gpurun_out/tests_i_tw.log 2>&1 || exit 1
: > gpurun_out/ab_i.jsonl
for L in libgw_engine.so libgw_engine_wg2.so libgw_engine_tw.so libgw_engine.so libgw_engine_wg2.so libgw_engine_tw.so; do
  GW_ENGINE_LIB=$B/$L timeout -k 10 200 python3 bench.py --workload rtt --steps 200 --warmup 5 --no-other --no-cpu-baseline \
      > gpurun_out/i_rtt.log 2>&1 || { tail -20 gpurun_out/i_rtt.log; exit 1; }
  echo "{\"lib\": \"$L\", \"line\": $(grep '^{' gpurun_out/i_rtt.log)}" >> gpurun_out/ab_i.jsonl
done
timeout -k 10 400 python3 tools/ab_headline.py $B/libgw_engine.so $B/libgw_engine_tw.so $B/libgw_engine_nogst.so $B/libgw_engine_cst.so \
    $B/libgw_engine.so $B/libgw_engine_tw.so $B/libgw_engine_nogst.so $B/libgw_engine_cst.so > gpurun_out/ab_head_i.jsonl 2> gpurun_out/ab_head_i.err || exit 1
bash tools/gpu_ab_r03g.sh
