"""Copy a rocprofv3 run (gpurun_out/prof_<tag>/) into profiles/ and derive the
per-launch HBM traffic of the step kernel from the PMC passes.

rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB per dispatch (derived from
TCC_EA0_RDREQ/WRREQ).  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads
half the bytes of 16-B-per-lane streaming loads; WRITE_SIZE is exact for
16-B-per-lane stores.  The step kernel's loads are mostly 4-8 B per lane
(uncalibrated widths), so the raw sum is reported together with the
algorithmic byte count; see DESIGN.md §Roofline.

usage: python tools/summarize_profile.py <tag> [kernel-substring]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short_name(n):
    """'void (anonymous namespace)::step_kernel<7>((anonymous namespace)::Params)'
    -> 'step_kernel<7>'"""
    n = n.replace('(anonymous namespace)::', '')
    if n.startswith('void '):
        n = n[5:]
    return n.split('(')[0][:60]


def main():
    tag = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else 'step_kernel'
    src = os.path.join(ROOT, 'gpurun_out', f'prof_{tag}')
    dst = os.path.join(ROOT, 'profiles')
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
    shutil.copy(stats, os.path.join(dst, f'{tag}_kernel_stats.csv'))
    rows = list(csv.DictReader(open(stats)))
    trace = list(csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_trace.csv'))))
    res = {}
    for r in trace:
        if kname in short_name(r['Kernel_Name']):
            res = {k: r.get(k, '') for k in ('LDS_Block_Size', 'Scratch_Size', 'VGPR_Count',
                                     'Accum_VGPR_Count', 'SGPR_Count', 'Workgroup_Size_X',
                                     'Grid_Size_X')}
            break
    pmc = {}
    for kind, counter in (('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE')):
        f = os.path.join(src, kind, 'run_counter_collection.csv')
        if not os.path.exists(f):
            continue
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter:
                vals[r['Kernel_Name']].append(float(r['Counter_Value']))
        for name, v in vals.items():
            if kname in name:
                pmc[counter] = sum(v) / len(v)
    lines = [f"# rocprofv3 summary `{tag}`", "",
             "Command: `rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py "
             "--no-cpu-baseline --no-other --steps 200 --warmup 20` (next_step auto-reset; PMC passes: `--pmc FETCH_SIZE` and "
             "`--pmc WRITE_SIZE`, separate runs, `--steps 30 --warmup 5`).", "",
             "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in rows[:8]:
        n = short_name(r['Name'])
        lines.append(f"| `{n}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                     f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | "
                     f"{float(r['Percentage']):.1f} |")
    lines += ["", f"{kname} resources: `{res}`", ""]
    out = {'tag': tag, 'kernel': kname, 'resources': res}
    if pmc:
        fetch_b = pmc.get('FETCH_SIZE', 0) * 1024
        write_b = pmc.get('WRITE_SIZE', 0) * 1024
        out.update(fetch_bytes_per_launch=fetch_b, write_bytes_per_launch=write_b,
                   hbm_bytes_per_launch=fetch_b + write_b)
        lines += [f"PMC per {kname} launch: FETCH_SIZE {fetch_b/1e6:.2f} MB, WRITE_SIZE "
                  f"{write_b/1e6:.2f} MB, sum {(fetch_b+write_b)/1e6:.2f} MB (raw, uncorrected)."]
    for r in rows:
        if kname in short_name(r['Name']):
            out['avg_ns'] = float(r['AverageNs'])
    json.dump(out, open(os.path.join(dst, f'pmc_{kname}.json'), 'w'), indent=1)
    open(os.path.join(dst, f'{tag}_summary.md'), 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


if __name__ == '__main__':
    main()
