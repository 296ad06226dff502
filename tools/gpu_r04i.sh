# placement checks + A/B against a previous build: bash tools/gpu_r04i.sh <lib.so>
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "oracle or golden or rollout or components or shard or builders" > gpurun_out/r04i_checks.log 2>&1 || { echo CHECKS FAIL; tail -30 gpurun_out/r04i_checks.log; exit 1; }
tail -1 gpurun_out/r04i_checks.log
B=abmarl_amd/_build/libgw_engine.so
bash tools/ab_closed.sh $B ${1:?lib} $B $1 || exit 1
timeout -k 10 400 python tools/ab_headline.py $B $1 $B $1 > gpurun_out/r04i_ab.jsonl 2>&1 || { echo AB FAIL; tail gpurun_out/r04i_ab.jsonl; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r04i_ab.jsonl'):
    d = json.loads(l); print(d['lib'][-26:], round(d['f20_ms'], 4), round(d['f100_ms'], 4))"
