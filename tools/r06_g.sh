#!/bin/bash
# Round 6, step G: config 4 workgroup-kernel variants vs HEAD (bd2: one-barrier
# counts, the observer's kept ballot on an existing barrier, the step-start
# table rebuild skipped when current; bd3: bd2 + the post-move tables updated
# in place instead of rebuilt): parity of the workgroup-kernel tests on bd3,
# then the rtt bench line alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
B=abmarl_amd/_build
P=$B/libgw_engine.so; T=$B/libgw_engine_bd2.so; D=$B/libgw_engine_bd3.so
GW_ENGINE_LIB=$D timeout -k 10 900 python -u -m pytest tests/test_engine_oracle.py tests/test_engine_golden.py tests/test_rollout.py tests/test_components.py tests/test_host_components.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1
rc=$?; tail -n1 $O/par.log; [ $rc -eq 0 ] || { echo "PARITY rc=$rc"; tail -30 $O/par.log; exit 1; }
AB_TAG=bd timeout -k 10 900 bash tools/ab_bench.sh rtt 100 $P $T $D $P $T $D $P $T $D || exit 1
cp gpurun_out/ab_bench_rtt_bd.jsonl $O/
python3 -c "
import json, collections
r = collections.defaultdict(list)
for l in open('$O/ab_bench_rtt_bd.jsonl'):
    d = json.loads(l); r[d['lib'].split('/')[-1]].append((round(d['line']['value'] / 1e9, 3), d['line']['roofline']['kernel_ms']))
for k, v in r.items(): print(k, v)"
