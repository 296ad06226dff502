#!/bin/bash
# Round 6, step C: closed-loop (one step launch per step) critical path:
# per-phase stamps incl. the serial attackers' sub-phases (stamps build), and
# the A/B of issue priority for envs that reset in the launch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python3 tools/stamps.py team_battle 4096 > $O/stamps_tb.log 2>&1 || { echo STAMPS FAIL; tail -20 $O/stamps_tb.log; exit 1; }
cat $O/stamps_tb.log
P=abmarl_amd/_build/libgw_engine.so; R=abmarl_amd/_build/libgw_engine_rprio.so
AB_TAG=closed_rprio AB_ARGS="--mode step" timeout -k 10 900 bash tools/ab_bench.sh team_battle 200 $P $R $P $R $P $R || exit 1
cp gpurun_out/ab_bench_team_battle_closed_rprio.jsonl $O/
python3 -c "
import json
for l in open('$O/ab_bench_team_battle_closed_rprio.jsonl'):
    d = json.loads(l); print(d['lib'][-28:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
# Pacman turn rollout: obs rows stored in whole 64-byte sectors (pacal) vs HEAD
A=abmarl_amd/_build/libgw_engine_pacal.so
AB_TAG=pacal timeout -k 10 900 bash tools/ab_bench.sh pacman 50 $P $A $P $A || exit 1
cp gpurun_out/ab_bench_pacman_pacal.jsonl $O/
python3 -c "
import json
for l in open('$O/ab_bench_pacman_pacal.jsonl'):
    d = json.loads(l); print(d['lib'][-28:], d['line']['value'], d['line']['roofline']['kernel_ms'])"
GW_ENGINE_LIB=$A timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 bench.py --gpus 1 --workload pacman --steps 50 --warmup 5 --no-other --no-cpu-baseline > $O/pw.log 2>&1 || { echo PMC FAIL; tail -20 $O/pw.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
o = sys.argv[1]
rows = [r for r in csv.DictReader(open(glob.glob(o + '/pw/**/*counter_collection.csv', recursive=True)[0]))
        if 'pac_kernel<4>' in r['Kernel_Name']]
per = {}
for r in rows:
    d = int(r['Dispatch_Id']); per[d] = per.get(d, 0.0) + float(r['Counter_Value'])
ds = sorted(per)
print('pac_kernel<4> dispatches', len(ds), 'timed (index 11) WRITE_SIZE bytes', per[ds[11]] * 1024.0)
PY
