"""Read off the memory instructions of every MT19937 twist-shaped block (the
0x9908b0df mask and the 25 instructions before it) per kernel of an ISA
listing: which address space reaches the key (ds_* = LDS-typed, flat_* =
generic pointer) and whether the key[i] / key[i + 1] pair is one 64-bit load.

    python tools/fault_r05/isa_diff.py <listing.s> [...]
"""
import collections
import re
import sys


def scan(path):
    cur = None
    twists = collections.Counter()
    lines = open(path).read().split('\n')
    for i, ln in enumerate(lines):
        m = re.match(r'^(_Z\S+|\.L_Z\S+):', ln)
        if m:
            cur = m.group(1)
            continue
        if '0x9908b0df' in ln:
            ops = sorted({x.strip().split()[0] for x in lines[max(0, i - 25):i]
                          if x.strip().startswith(('flat_', 'ds_', 'global_', 'scratch_'))})
            twists[(cur, tuple(ops))] += 1
    return twists


if __name__ == '__main__':
    for path in sys.argv[1:]:
        print('==', path)
        for (k, ops), n in sorted(scan(path).items()):
            k = re.sub(r'^_ZN12_GLOBAL__N_1\d+', '', k or '?')
            print(f'  {k[:48]:48s} x{n:<3d} {" ".join(ops)}')
