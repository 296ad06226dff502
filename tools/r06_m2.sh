#!/bin/bash
# Round 6, step M2: config 4 with the hidden-byte masks spread from 4 bits at a
# possible candidate in the attacker's window: (True, []) after one count
# barrier instead of the mask / list / damage passes): parity of the
# workgroup-kernel tests, then the rtt line alternating with production.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m2
mkdir -p $O
B=abmarl_amd/_build
P=$B/libgw_engine.so; D=$B/libgw_engine_mask.so
GW_ENGINE_LIB=$D timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py tests/test_rollout.py tests/test_components.py tests/test_host_components.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1
rc=$?; tail -n1 $O/par.log; [ $rc -eq 0 ] || { echo "PARITY rc=$rc"; tail -30 $O/par.log; exit 1; }
AB_TAG=mask timeout -k 10 900 bash tools/ab_bench.sh rtt 100 $P $D $P $D $P $D || exit 1
cp gpurun_out/ab_bench_rtt_mask.jsonl $O/
python3 -c "
import json, collections
r = collections.defaultdict(list)
for l in open('$O/ab_bench_rtt_mask.jsonl'):
    d = json.loads(l); r[d['lib'].split('/')[-1]].append((round(d['line']['value'] / 1e9, 3), d['line']['roofline']['kernel_ms']))
for k, v in r.items(): print(k, v)"
