# round-4: Pacman / config-4 checks and quick lines: bash tools/gpu_r04e.sh
set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
GW_ENGINE_VARIANT=checks timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pacman or turn or f3 or rtt or reach or workgroup" > gpurun_out/r04e_checks.log 2>&1 || { echo CHECKS FAIL; tail -30 gpurun_out/r04e_checks.log; exit 1; }
tail -1 gpurun_out/r04e_checks.log
timeout -k 10 300 python -c "
import bench, json
print(json.dumps({k: bench.quick_config(k) for k in ('pacman', 'rtt', 'rtt_8192')}))" > gpurun_out/r04e_quick.json 2>&1 || { echo QUICK FAIL; tail -20 gpurun_out/r04e_quick.json; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/r04e_quick.json').read().strip().splitlines()[-1])
for k, v in d.items():
    r = v['rollout'] or {}
    print(k, v['value'], v['kernel_ms'], '| rollout', r.get('value'), r.get('launch_ms'), r.get('achieved_GBs'))"
