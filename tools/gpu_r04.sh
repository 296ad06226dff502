# round-4 GPU checks: bash tools/gpu_r04.sh [tests|perf1|perf2|all]
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
if [ "${1:-all}" != perf1 ] && [ "${1:-all}" != perf2 ]; then
GW_ENGINE_VARIANT=checks timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ammo or shard or registry or builders or components or golden or oracle or known or rollout" > gpurun_out/r04_checks.log 2>&1 || { echo CHECKS FAIL; tail -40 gpurun_out/r04_checks.log; exit 1; }
tail -2 gpurun_out/r04_checks.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_gputest.log 2>&1 || { echo TESTS FAIL; tail -40 gpurun_out/r04_gputest.log; exit 1; }
tail -2 gpurun_out/r04_gputest.log
[ "${1:-all}" = tests ] && exit 0
fi
if [ "${1:-all}" != perf2 ]; then
timeout -k 10 600 python tools/ab_headline.py abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_keypre0.so abmarl_amd/_build/libgw_engine_keypre2.so abmarl_amd/_build/libgw_engine_jacobi.so abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_keypre0.so abmarl_amd/_build/libgw_engine_keypre2.so abmarl_amd/_build/libgw_engine_jacobi.so > gpurun_out/r04_ab_place.jsonl 2>&1 || { echo AB FAIL; tail gpurun_out/r04_ab_place.jsonl; exit 1; }
cut -c1-200 gpurun_out/r04_ab_place.jsonl
AB_ARGS="--mode step" AB_TAG=closed timeout -k 10 900 bash tools/ab_bench.sh team_battle 200 abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_keypre0.so abmarl_amd/_build/libgw_engine_keypre2.so abmarl_amd/_build/libgw_engine_jacobi.so abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_keypre0.so abmarl_amd/_build/libgw_engine_keypre2.so abmarl_amd/_build/libgw_engine_jacobi.so || { echo AB CLOSED FAIL; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ab_bench_team_battle_closed.jsonl'):
    d = json.loads(l); print(d['lib'][-28:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_bench20.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r04_bench20.log; exit 1; }
tail -1 gpurun_out/r04_bench20.log | cut -c1-400
[ "${1:-all}" = perf1 ] && exit 0
fi
timeout -k 10 240 python bench.py --workload rtt --steps 200 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/r04_bench_rtt.log 2>&1 || { echo RTT FAIL; tail -20 gpurun_out/r04_bench_rtt.log; exit 1; }
tail -1 gpurun_out/r04_bench_rtt.log | cut -c1-400
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r04_stamps_tb.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r04_stamps_tb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_stamps_tb.log | tail -25
timeout -k 10 600 bash tools/ab_bench.sh rtt 200 abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_wgserial.so abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_wgserial.so || { echo AB RTT FAIL; exit 1; }
cut -c1-300 gpurun_out/ab_bench_rtt.jsonl
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r04_stamps_rtt.log 2>&1 || { echo STAMPS RTT FAIL; tail -20 gpurun_out/r04_stamps_rtt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_stamps_rtt.log | tail -25
timeout -k 10 600 bash tools/ab_bench.sh pacman 200 abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_pacold.so abmarl_amd/_build/libgw_engine.so abmarl_amd/_build/libgw_engine_pacold.so || { echo AB PAC FAIL; exit 1; }
cut -c1-300 gpurun_out/ab_bench_pacman.jsonl
