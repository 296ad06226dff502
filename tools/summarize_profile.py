"""Summarize tools/profile.sh output into profiles/<tag>_*:

  <tag>_<wl>_kernel_stats.csv   rocprofv3 --stats table (copied)
  <tag>_<wl>_summary.md         per-kernel calls / avg / min / max / share,
                                the step kernel's resources, PMC traffic
  pmc_<kernel>.json             FETCH_SIZE / WRITE_SIZE per step launch:
                                raw (KiB -> bytes) and the gfx950-corrected
                                HBM bytes (MI355X_MICROARCH.md §HBM: FETCH_SIZE
                                reports half the bytes of coalesced reads, so
                                it is doubled; WRITE_SIZE is exact for 16-B
                                stores) -- bench.py reports hbm_bytes_per_launch
                                as roofline.traffic.

usage: python tools/summarize_profile.py <tag> <team_battle|rtt|maze> --mode rollout|step --raw DIR --dest DIR
(rollout mode: every step-kernel dispatch is a gw_rollout fragment of
--fragment steps; the json is pmc_<kernel>_rollout_f<fragment>.json)
"""
import argparse
import csv
import glob
import json
import os
import shutil

KERNEL = {'team_battle': 'step_kernel<7, 1>', 'rtt': 'wg_step_kernel<7>', 'maze': 'lane_step_kernel<5, 10>'}


def find(root, pattern):
    hits = sorted(glob.glob(os.path.join(root, '**', pattern), recursive=True))
    if not hits:
        raise SystemExit(f'no {pattern} under {root}')
    return hits[0]


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0][:60]


def pmc_per_launch(root, counter, kernel):
    path = find(root, '*counter_collection.csv')
    vals = []
    for row in csv.DictReader(open(path)):
        if row.get('Counter_Name') != counter:
            continue
        if short(row['Kernel_Name']) != kernel:
            continue
        vals.append(float(row['Counter_Value']))
    if not vals:
        raise SystemExit(f'{counter}: no {kernel} dispatches in {path}')
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('tag')
    ap.add_argument('workload', choices=list(KERNEL))
    ap.add_argument('--raw', required=True)
    ap.add_argument('--dest', required=True)
    ap.add_argument('--mode', default='step', choices=['step', 'rollout'])
    ap.add_argument('--stats-args', default='--steps 200 --warmup 20')
    ap.add_argument('--pmc-args', default='--steps 30 --warmup 5')
    ap.add_argument('--fragment', type=int, default=100)
    a = ap.parse_args()
    kernel = KERNEL[a.workload]
    os.makedirs(a.dest, exist_ok=True)
    sroot = os.path.join(a.raw, f'prof_{a.tag}_stats')
    stats = find(sroot, '*kernel_stats.csv')
    suffix = f'_rollout_f{a.fragment}' if a.mode == 'rollout' else ''
    base = f'{a.tag}_{a.workload}' + suffix
    shutil.copy(stats, os.path.join(a.dest, base + '_kernel_stats.csv'))
    rows = list(csv.DictReader(open(stats)))
    res = {}
    try:
        trace = find(sroot, '*kernel_trace.csv')
        for r in csv.DictReader(open(trace)):
            if short(r['Kernel_Name']) == kernel:
                res = {k: r[k] for k in ('LDS_Block_Size', 'Scratch_Size', 'VGPR_Count', 'Accum_VGPR_Count',
                                         'SGPR_Count', 'Workgroup_Size_X', 'Grid_Size_X') if k in r}
                break
    except SystemExit:
        pass
    fetch_kib, nf = pmc_per_launch(os.path.join(a.raw, f'prof_{a.tag}_FETCH_SIZE'), 'FETCH_SIZE', kernel)
    write_kib, nw = pmc_per_launch(os.path.join(a.raw, f'prof_{a.tag}_WRITE_SIZE'), 'WRITE_SIZE', kernel)
    fetch, write = fetch_kib * 1024.0, write_kib * 1024.0
    avg_ns = next(float(r['AverageNs']) for r in rows if short(r['Name']) == kernel)
    pmc = {'tag': a.tag, 'kernel': kernel, 'resources': res,
           'fetch_bytes_per_launch_raw': fetch, 'write_bytes_per_launch': write,
           'fetch_bytes_per_launch_corrected': 2.0 * fetch,
           'hbm_bytes_per_launch': 2.0 * fetch + write,
           'hbm_bytes_per_launch_raw': fetch + write,
           'dispatches': {'FETCH_SIZE': nf, 'WRITE_SIZE': nw}, 'avg_ns': avg_ns,
           'rocprof_avg_ms': avg_ns / 1e6, 'mode': a.mode,
           'steps_per_launch': a.fragment if a.mode == 'rollout' else 1}
    json.dump(pmc, open(os.path.join(a.dest, f'pmc_{kernel.split("<")[0]}{suffix}.json'), 'w'), indent=1)
    lines = [f'# rocprofv3 summary `{a.tag}` ({a.workload})', '',
             f'Command: `rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py '
             f'--workload {a.workload} --mode {a.mode} --no-cpu-baseline --no-other --fragment {a.fragment} '
             f'{a.stats_args}`; PMC: `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE`, separate runs, '
             f'`{a.pmc_args}` (tools/profile.sh).' +
             (f' Every step-kernel dispatch is a {a.fragment}-step gw_rollout fragment.' if a.mode == 'rollout' else ''),
             '',
             '| kernel | calls | avg us | min us | max us | % |', '|---|---|---|---|---|---|']
    for r in rows:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.1f} |")
    lines += ['', f'{kernel} resources: `{res}`', '',
              f'PMC per {kernel} launch: FETCH_SIZE {fetch / 1e6:.2f} MB raw '
              f'(x2 gfx950 correction: {2 * fetch / 1e6:.2f} MB), WRITE_SIZE {write / 1e6:.2f} MB; '
              f'HBM traffic {pmc["hbm_bytes_per_launch"] / 1e6:.2f} MB corrected '
              f'({pmc["hbm_bytes_per_launch_raw"] / 1e6:.2f} MB raw).']
    open(os.path.join(a.dest, base + '_summary.md'), 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


if __name__ == '__main__':
    main()
