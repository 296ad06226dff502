# A/B of engine builds on config 5 (Pacman, TurnBasedManager, 16384 envs):
#   bash tools/ab_pac.sh <lib.so> ...   (turn rollout and per-turn launches)
set -o pipefail
timeout -k 10 600 bash tools/ab_bench.sh pacman 200 "$@" || exit 1
AB_TAG=turn AB_ARGS="--mode step" timeout -k 10 600 bash tools/ab_bench.sh pacman 200 "$@" || exit 1
python3 -c "
import json
for f in ('gpurun_out/ab_bench_pacman.jsonl', 'gpurun_out/ab_bench_pacman_turn.jsonl'):
    for l in open(f):
        d = json.loads(l); print(f[-12:], d['lib'][-28:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
