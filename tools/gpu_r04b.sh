# round-4 measurements of HEAD: bash tools/gpu_r04b.sh [a|b]
#  a: the driver's command, the closed loop, stamps and the tail probe of
#     the headline kernel, config 4 (rtt) line + A/B + stamps
#  b: Pacman A/B, the strong-scaling proxy (with the multi-wave variant)
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
B=abmarl_amd/_build/libgw_engine
if [ "${1:-a}" = a ]; then
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04b_bench20.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r04b_bench20.log; exit 1; }
tail -1 gpurun_out/r04b_bench20.log | cut -c1-300
timeout -k 10 240 python bench.py --mode step --steps 200 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/r04b_closed.log 2>&1 || { echo CLOSED FAIL; tail -20 gpurun_out/r04b_closed.log; exit 1; }
python3 -c "
import json; d = json.loads(open('gpurun_out/r04b_closed.log').read().strip().splitlines()[-1]); print('closed', d['value'], d['roofline']['kernel_ms'])"
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r04b_stamps_tb.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r04b_stamps_tb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04b_stamps_tb.log | tail -32
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/tail_probe.py --frag 20 > gpurun_out/r04b_tail_probe.log 2>&1 || { echo TAIL FAIL; tail -20 gpurun_out/r04b_tail_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04b_tail_probe.log | head -20
timeout -k 10 240 python bench.py --workload rtt --steps 200 --warmup 5 --no-other --no-cpu-baseline > gpurun_out/r04b_bench_rtt.log 2>&1 || { echo RTT FAIL; tail -20 gpurun_out/r04b_bench_rtt.log; exit 1; }
tail -1 gpurun_out/r04b_bench_rtt.log | cut -c1-300
timeout -k 10 600 bash tools/ab_bench.sh rtt 200 $B.so ${B}_wgserial.so $B.so ${B}_wgserial.so || { echo AB RTT FAIL; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ab_bench_rtt.jsonl'):
    d = json.loads(l); print(d['lib'][-26:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py rtt > gpurun_out/r04b_stamps_rtt.log 2>&1 || { echo STAMPS RTT FAIL; tail -20 gpurun_out/r04b_stamps_rtt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04b_stamps_rtt.log | tail -25
fi
if [ "${1:-a}" = b ]; then
timeout -k 10 600 bash tools/ab_bench.sh pacman 200 $B.so ${B}_pacold.so $B.so ${B}_pacold.so || { echo AB PAC FAIL; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ab_bench_pacman.jsonl'):
    d = json.loads(l); print(d['lib'][-26:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
timeout -k 10 900 bash tools/strong_proxy.sh || { echo PROXY FAIL; exit 1; }
fi
