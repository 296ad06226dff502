"""Summarize tools/prof_headline.sh output (the driver's headline workload:
bench.py --gpus 1 --steps 20 --warmup 5) into

  <dest>/<tag>_headline_kernel_stats.csv   rocprofv3 --stats table (copied)
  <dest>/<tag>_headline_summary.md         per-dispatch durations of the
      headline run's step_kernel launches (pre-roll fragments, the last
      untimed 20-step fragment, THE timed launch), the idle gap before the
      timed launch, the events / host figures of the same run, PMC traffic
      and SQ counters of the timed launch
  <dest>/pmc_step_kernel_rollout_f20.json  what bench.py reads for
      roofline.traffic / traffic_ratio / rocprof_kernel_ms

Dispatch order: bench.py's run_rollout launches the pre-roll + warmup
(1005 steps) as fragments of 100 steps, the last one exactly 20 steps, then
the timed 20-step launch; so in the first engine's run the step_kernel
dispatches are [100] * 9 + [85, 20] and then the timed one (index 11).

--workload rtt: the same for BASELINE config 4's line (bench.py --workload
rtt --steps 100 --warmup 5: wg_step_kernel<7>, 1024 envs, one timed 100-step
launch; <tag>_rtt_* and pmc_wg_step_kernel_rollout_f100.json).
--workload pacman: config 5 (bench.py --workload pacman --steps 50 --warmup
5: pac_kernel<4>, 16384 envs, one timed 50-turn gw_turn_rollout launch;
<tag>_pacman_* and pmc_pac_kernel_rollout_f50.json; algorithmic bytes =
bench.pacman_turn_rollout_bytes of that launch).

usage: python tools/summarize_headline.py <tag> --raw DIR --dest DIR [--workload rtt]
"""
import argparse
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# workload: (kernel, envs, entity slots, obs side, fragment steps, action ints
# per slot, bench.py arguments)
WORKLOADS = {
    'team_battle': ('step_kernel<7, 1>', 4096, 64, 7, 20, 3, '--gpus 1 --steps 20 --warmup 5'),
    'rtt': ('wg_step_kernel<7>', 1024, 256, 7, 100, 11, '--gpus 1 --workload rtt --steps 100 --warmup 5'),
    # config 5: pac_kernel<PAC_STEP_TURN>, one timed 50-turn gw_turn_rollout
    # (lanes and food words from the bench line's config)
    'pacman': ('pac_kernel<4>', 16384, None, None, 50, 2, '--gpus 1 --workload pacman --steps 50 --warmup 5'),
}
KERNEL = 'step_kernel<7, 1>'
E, A, S, F, ACT_DIM = 4096, 64, 7, 20, 3
BENCH_ARGS = WORKLOADS['team_battle'][6]


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0]


def fragments(preroll=1000, warmup=5, fragment=100, steps=F):
    """bench.run_rollout's untimed fragment sizes (the timed one follows)."""
    Fr = max(1, min(fragment, steps))
    nfrag = max(Fr, min(fragment, max(preroll + warmup, 1)))
    sizes, rest = [], preroll + warmup
    last = min(Fr, rest)
    rest -= last
    while rest > 0:
        sizes.append(min(nfrag, rest))
        rest -= sizes[-1]
    if last:
        sizes.append(last)
    return sizes


def find(root, pattern):
    hits = sorted(glob.glob(os.path.join(root, '**', pattern), recursive=True))
    if not hits:
        raise SystemExit(f'no {pattern} under {root}')
    return hits[0]


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith('{"metric"'):
            return json.loads(line)
    raise SystemExit(f'no bench JSON line in {log}')


def trace(root):
    rows = list(csv.DictReader(open(find(root, '*kernel_trace.csv'))))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    return rows


def counters(root):
    """{counter: [value per step_kernel dispatch, in dispatch order]}"""
    rows = list(csv.DictReader(open(find(root, '*counter_collection.csv'))))
    per = {}
    for r in rows:
        if short(r['Kernel_Name']) != KERNEL:
            continue
        per.setdefault(r['Counter_Name'], {})
        d = int(r['Dispatch_Id'])
        per[r['Counter_Name']][d] = per[r['Counter_Name']].get(d, 0.0) + float(r['Counter_Value'])
    return {k: [v[d] for d in sorted(v)] for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('tag')
    ap.add_argument('--raw', required=True)
    ap.add_argument('--dest', required=True)
    ap.add_argument('--workload', default='team_battle', choices=sorted(WORKLOADS))
    a = ap.parse_args()
    global KERNEL, E, A, S, F, ACT_DIM, BENCH_ARGS
    KERNEL, E, A, S, F, ACT_DIM, BENCH_ARGS = WORKLOADS[a.workload]
    kind = 'headline' if a.workload == 'team_battle' else a.workload
    from bench import rollout_bytes
    os.makedirs(a.dest, exist_ok=True)
    sizes = fragments(steps=F)
    ti = len(sizes)                          # index of the timed dispatch
    st = os.path.join(a.raw, 'stats')
    shutil.copy(find(st, '*kernel_stats.csv'), os.path.join(a.dest, f'{a.tag}_{kind}_kernel_stats.csv'))
    line = bench_line(os.path.join(a.raw, 'stats.log'))
    rows = trace(st)
    sk = [i for i, r in enumerate(rows) if short(r['Kernel_Name']) == KERNEL]
    dur = lambda i: (int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3
    timed, prev_frag = sk[ti], sk[ti - 1]
    # idle gap: the timed launch's start after the end of the previous GPU op
    gap = (int(rows[timed]['Start_Timestamp']) - int(rows[timed - 1]['End_Timestamp'])) / 1e3
    prev_name = short(rows[timed - 1]['Kernel_Name'])
    # the second engine (same_step) repeats the pattern right after
    timed2 = sk[2 * ti + 1] if len(sk) > 2 * ti + 1 else None
    res = {k: rows[timed][k] for k in ('LDS_Block_Size', 'Scratch_Size', 'VGPR_Count', 'Accum_VGPR_Count',
                                       'SGPR_Count', 'Workgroup_Size_X', 'Grid_Size_X') if k in rows[timed]}
    # PMC passes (the short command: the first engine's run only)
    p = {}
    for d in sorted(glob.glob(os.path.join(a.raw, 'p[0-9]*'))):
        if os.path.isdir(d):
            for k, v in counters(d).items():
                p[k] = v
    pl = bench_line(os.path.join(a.raw, 'p1.log'))
    acting = pl['acting_agent_steps']
    if a.workload == 'pacman':
        from bench import pacman_turn_rollout_bytes
        A = pl['config']['lanes']
        pw = (pl['config']['passive_entities'] + 31) // 32
        HW = pl['config']['cells']
        # every acting agent-step returns one observation row (bench.py)
        alg = pacman_turn_rollout_bytes(E, A, HW, pw, F, acting)
        alg_writes = F * E * (A * (8 + 1 + 1) + 1 + 4) + 4 * HW * acting + E * (A * 29 + 4 * pw + 4 + 4 + 8 + 8)
        rb = 'bench.pacman_turn_rollout_bytes'
    else:
        alg = rollout_bytes(E, A, S, F, acting, ACT_DIM)
        alg_writes = F * E * (A * (8 + 1) + 1) + 4 * S * S * acting + E * A * (8 + 4 + 8 + 1) + E * 41
        rb = 'bench.rollout_bytes'
    fetch = p['FETCH_SIZE'][ti] * 1024.0
    write = p['WRITE_SIZE'][ti] * 1024.0
    hbm = 2.0 * fetch + write
    sq = {k: v[ti] for k, v in p.items() if k.startswith('SQ_')}
    waves = sq.get('SQ_WAVES') or 1.0
    pmc = {
        'tag': a.tag, 'kernel': KERNEL, 'envs': E,
        'workload_args': f'bench.py {BENCH_ARGS} (--no-other --no-cpu-baseline for '
                         f'the PMC passes): 1000-step pre-roll, the timed {F}-step gw_rollout launch',
        'dispatch_index': ti, 'resources': res,
        'acting_agent_steps': acting,
        'algorithmic_bytes_per_launch': alg,
        'algorithmic_write_bytes_per_launch': alg_writes,
        'fetch_bytes_per_launch_raw': fetch, 'fetch_bytes_per_launch_corrected': 2.0 * fetch,
        'write_bytes_per_launch': write,
        'hbm_bytes_per_launch': hbm,
        'traffic_ratio': hbm / alg, 'write_ratio': write / alg_writes,
        'rocprof_timed_dispatch_ms': dur(timed) / 1e3,
        'rocprof_avg_ms': dur(timed) / 1e3,
        'rocprof_prev_fragment_ms': dur(prev_frag) / 1e3,
        'steps_per_launch': F, 'mode': 'rollout',
        'sq_timed_launch': sq,
    }
    json.dump(pmc, open(os.path.join(a.dest, f'pmc_{KERNEL.split("<")[0]}_rollout_f{F}.json'), 'w'), indent=1)
    roof = line.get('roofline', {})
    L = [f'# {kind} profile `{a.tag}`' + (': the driver\'s workload' if kind == 'headline' else ''), '',
         'Command (kernel trace): `rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py '
         f'{BENCH_ARGS}`; PMC: one `--pmc` pass per counter set, the same command with '
         '`--no-other --no-cpu-baseline` (tools/prof_headline.sh).', '',
         f'## {KERNEL} dispatches of the headline engine (stats run)', '',
         '| # | steps | duration us |', '|---|---|---|']
    for k, i in enumerate(sk[:ti + 1]):
        L.append(f'| {k} | {sizes[k] if k < ti else str(F) + " (TIMED)"} | {dur(i):.1f} |')
    L += ['',
          f'- timed launch: **{dur(timed):.1f} us** (rocprof); the untimed {F}-step launch right before it: '
          f'{dur(prev_frag):.1f} us; the same_step engine\'s timed launch: '
          f'{(dur(timed2) if timed2 is not None else float("nan")):.1f} us',
          f'- idle gap before the timed launch (after `{prev_name}` ended): {gap:.1f} us '
          '(host: synchronize, acting read-back, synchronize, event record, launch)',
          f'- the same run\'s HIP-event launch time (bench line `roofline.kernel_ms`): '
          f'{roof.get("kernel_ms")} ms; '
          f'wall ms_per_step x {F}: {line.get("ms_per_step", 0) * F:.4f} ms; value {line.get("value"):.4g}',
          f'- resources: `{res}`', '',
          '## Traffic of the timed launch (PMC run)', '',
          f'- acting agent-steps in the launch: {acting}',
          f'- algorithmic bytes ({rb}): {alg / 1e6:.2f} MB '
          f'({alg / acting:.1f} B per acting agent-step)',
          f'- FETCH_SIZE {fetch / 1e6:.2f} MB raw, x2 gfx950 correction {2 * fetch / 1e6:.2f} MB; '
          f'WRITE_SIZE {write / 1e6:.2f} MB (algorithmic writes {alg_writes / 1e6:.2f} MB: '
          f'ratio {write / alg_writes:.3f})',
          f'- HBM traffic {hbm / 1e6:.2f} MB = **{hbm / alg:.3f}x** the algorithmic bytes', '',
          '## SQ counters of the timed launch (per wave = per env)', '',
          '| counter | launch total | per wave |', '|---|---|---|']
    for k in sorted(sq):
        L.append(f'| {k} | {sq[k]:.0f} | {sq[k] / waves:.1f} |')
    if 'SQ_LDS_BANK_CONFLICT' in sq and sq.get('SQ_LDS_IDX_ACTIVE'):
        L += ['', f'LDS bank conflicts / LDS-active cycles: '
                  f'{sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"]:.3f}']
    if 'SQ_WAIT_ANY' in sq and sq.get('SQ_WAVE_CYCLES'):
        L += [f'wave cycles waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES): {sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]:.3f}']
    open(os.path.join(a.dest, f'{a.tag}_{kind}_summary.md'), 'w').write('\n'.join(L) + '\n')
    print('\n'.join(L))


if __name__ == '__main__':
    main()
