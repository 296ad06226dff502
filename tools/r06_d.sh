#!/bin/bash
# Round 6, step D: WRITE_SIZE calibration of the Pacman store patterns
# (tools/wsize_calib.hip) and the closed-loop stamps with the serial
# attackers' sub-phases accumulated in registers.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib -o run -- tools/bin/wsize_calib > $O/calib.log 2>&1 || { echo CALIB FAIL; tail -20 $O/calib.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, re
o = sys.argv[1]
known = {}
for line in open(o + '/calib.log'):
    m = re.match(r'(k_\w+) bytes (\d+)', line)
    if m:
        known[m.group(1)] = int(m.group(2))
per = {}
for r in csv.DictReader(open(glob.glob(o + '/calib/**/*counter_collection.csv', recursive=True)[0])):
    k = r['Kernel_Name'].split('(')[0].replace('void ', '').strip()
    per.setdefault(k, {}).setdefault(int(r['Dispatch_Id']), 0.0)
    per[k][int(r['Dispatch_Id'])] += float(r['Counter_Value']) * 1024.0
for k, d in per.items():
    vals = [d[i] for i in sorted(d)]
    kb = known.get(k)
    print(k, 'WRITE_SIZE per dispatch', [round(v / 1e6, 2) for v in vals], 'MB; known', kb / 1e6 if kb else None,
          'MB; factor', [round(v / kb, 4) for v in vals] if kb else None)
PY
GW_ENGINE_VARIANT=stamps timeout -k 10 300 python3 tools/stamps.py team_battle 4096 > $O/stamps_tb.log 2>&1 || { echo STAMPS FAIL; tail -20 $O/stamps_tb.log; exit 1; }
grep -A12 "serial attack_one" $O/stamps_tb.log; tail -4 $O/stamps_tb.log
