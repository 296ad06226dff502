# closed-loop (one step launch per step) A/B of engine builds on the headline:
#   bash tools/ab_closed.sh <lib.so> ...
set -o pipefail
AB_ARGS="--mode step" AB_TAG=closed timeout -k 10 900 bash tools/ab_bench.sh team_battle 200 "$@" || exit 1
python3 -c "
import json
for l in open('gpurun_out/ab_bench_team_battle_closed.jsonl'):
    d = json.loads(l); print(d['lib'][-28:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
