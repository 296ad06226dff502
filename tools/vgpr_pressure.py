"""Live VGPRs per source location of one kernel, from LLVM's post-RA MIR
(hipcc ... -mllvm -print-after=virtregrewriter -mllvm -filter-print-funcs=K
2> mir.txt).

Backward liveness inside each block from its successors' liveins.  Prints the
source lines where the live 32-bit VGPR count is within `slack` of the peak
(with their inlined call chains), and the maximum per call site of the
kernel body.  Used to find what holds wg_step_kernel<7>'s registers
(DESIGN §4, config 4 in one dispatch round).

usage: python tools/vgpr_pressure.py mir.txt [slack]"""
import collections
import re
import sys

REG = re.compile(r'\$(vgpr\d+(?:_vgpr\d+)*)')
IDEF = re.compile(r'implicit-def (?:dead )?\$(\S+)')


def units(tok):
    return tok.split('_')


def analyze(path):
    """[(live VGPRs before the instruction, its debug location)]"""
    dump = open(path).read().split('# *** IR Dump After')[-1]
    blocks, order, cur = {}, [], None
    for ln in dump.split('\n'):
        s = ln.strip()
        m = re.match(r'^(?:\d+B\s+)?bb\.(\d+)\b.*:$', s)
        if m:
            cur = int(m.group(1))
            blocks[cur] = {'succ': [], 'livein': set(), 'ins': []}
            order.append(cur)
            continue
        if cur is None:
            continue
        if s.startswith('successors:'):
            blocks[cur]['succ'] = [int(x) for x in re.findall(r'%bb\.(\d+)', s)]
        elif s.startswith('liveins:'):
            for tok in REG.findall(s):
                blocks[cur]['livein'].update(units(tok))
        elif re.match(r'^\d+B\s', s):
            blocks[cur]['ins'].append(s)
    out = []
    for b in order:
        live = set()
        for sb in blocks[b]['succ']:
            live |= blocks[sb]['livein']
        for ins in reversed(blocks[b]['ins']):
            body, _, loc = ins.partition('; ')
            body = re.sub(r'^\d+B\s+', '', body)
            lhs, eq, rhs = body.partition(' = ')
            if not eq:
                lhs, rhs = '', body
            defs = set(u for t in REG.findall(lhs) for u in units(t))
            defs |= set(u for t in IDEF.findall(rhs) if t.startswith('vgpr') for u in units(t))
            uses = set(u for t in REG.findall(IDEF.sub('', rhs)) for u in units(t))
            live -= defs
            live |= uses
            out.append((len(live), loc.strip()))
    return out


def strip_cols(loc):
    return re.sub(r'(:\d+):\d+', r'\1', loc)


def main(path, slack=8):
    rows = analyze(path)
    mx = max(n for n, _ in rows)
    print('max live VGPRs', mx)
    agg = collections.Counter()
    for n, loc in rows:
        if n >= mx - slack:
            agg[strip_cols(loc)[:300]] += 1
    for k, v in agg.most_common(30):
        print(f'{v:5d}  {k}')
    # per call site of the kernel body: the outermost frame
    site = collections.defaultdict(int)
    for n, loc in rows:
        frames = re.findall(r'([\w./]+:\d+)', strip_cols(loc))
        key = ' <- '.join(frames[-2:][::-1]) if frames else '?'
        site[key] = max(site[key], n)
    print('\nmax live per (outermost, next) frame, top 30:')
    for k, v in sorted(site.items(), key=lambda kv: -kv[1])[:30]:
        print(f'{v:5d}  {k}')


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
