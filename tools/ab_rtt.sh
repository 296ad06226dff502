# A/B of engine builds on config 4 at 1024 and 8192 envs:
#   bash tools/ab_rtt.sh <lib.so> <lib.so>   (each twice at 1024, once at 8192)
set -o pipefail
A=${1:?lib}; B=${2:?lib}
timeout -k 10 600 bash tools/ab_bench.sh rtt 200 $A $B $A $B || exit 1
AB_TAG=8192 AB_ARGS="--envs 8192" timeout -k 10 600 bash tools/ab_bench.sh rtt 100 $A $B || exit 1
python3 -c "
import json
for f in ('gpurun_out/ab_bench_rtt.jsonl', 'gpurun_out/ab_bench_rtt_8192.jsonl'):
    for l in open(f):
        d = json.loads(l); print(f[-10:], d['lib'][-28:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
