# round-4 quick check of HEAD: bash tools/gpu_r04f.sh
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pacman or turn or f3 or oracle or rollout" > gpurun_out/r04f_checks.log 2>&1 || { echo CHECKS FAIL; tail -30 gpurun_out/r04f_checks.log; exit 1; }
tail -1 gpurun_out/r04f_checks.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04f_bench20.log 2>&1 || { echo BENCH FAIL; tail -20 gpurun_out/r04f_bench20.log; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/r04f_bench20.log').read().strip().splitlines()[-1])
print('headline', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], 'closed', d['closed_loop']['value'], d['closed_loop']['kernel_ms'])
for k, v in d['other_configs'].items():
    r = v['rollout'] or {}
    print(k, v['value'], v['kernel_ms'], '| rollout', r.get('value'), r.get('launch_ms'))"
