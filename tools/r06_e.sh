#!/bin/bash
# Round 6, step E: headline (driver's command: 20 timed steps after a
# 1000-step pre-roll) A/B of step_kernel<7,1> builds: HEAD vs no MachineLICM
# (nolicm), the lane index re-derived per step (laund), both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
B=abmarl_amd/_build
P=$B/libgw_engine.so; N=$B/libgw_engine_nolicm.so; L=$B/libgw_engine_laund.so; X=$B/libgw_engine_both.so
AB_TAG=head timeout -k 10 1000 bash tools/ab_bench.sh team_battle 20 $P $N $L $X $P $N $L $X $P $N $L $X || exit 1
cp gpurun_out/ab_bench_team_battle_head.jsonl $O/
python3 -c "
import json, collections
r = collections.defaultdict(list)
for l in open('$O/ab_bench_team_battle_head.jsonl'):
    d = json.loads(l); r[d['lib'].split('/')[-1]].append((round(d['line']['value'] / 1e9, 3), d['line']['roofline']['kernel_ms']))
for k, v in r.items(): print(k, v)"
