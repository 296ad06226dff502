# round-4 placement A/B: bash tools/gpu_r04c.sh <variant-name>
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
B=abmarl_amd/_build/libgw_engine
V=${1:?variant}
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "oracle or golden or rollout or components or shard" > gpurun_out/r04c_checks.log 2>&1 || { echo CHECKS FAIL; tail -30 gpurun_out/r04c_checks.log; exit 1; }
tail -1 gpurun_out/r04c_checks.log
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python tools/stamps.py team_battle > gpurun_out/r04c_stamps_tb.log 2>&1 || { echo STAMPS FAIL; tail -20 gpurun_out/r04c_stamps_tb.log; exit 1; }
grep -A30 "resetting envs" gpurun_out/r04c_stamps_tb.log | head -16
timeout -k 10 600 python tools/ab_headline.py $B.so ${B}_$V.so $B.so ${B}_$V.so > gpurun_out/r04c_ab.jsonl 2>&1 || { echo AB FAIL; tail gpurun_out/r04c_ab.jsonl; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r04c_ab.jsonl'):
    d = json.loads(l); print(d['lib'][-26:], round(d['f20_ms'], 4), round(d['f100_ms'], 4))"
AB_ARGS="--mode step" AB_TAG=closed timeout -k 10 600 bash tools/ab_bench.sh team_battle 200 $B.so ${B}_$V.so $B.so ${B}_$V.so || { echo AB CLOSED FAIL; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ab_bench_team_battle_closed.jsonl'):
    d = json.loads(l); print(d['lib'][-26:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
