"""Build the production engine of a given commit (or of the working tree's
sources with a list of -D flags) into abmarl_amd/_build/ab/<name>/, for
in-call A/B runs against HEAD (GW_ENGINE_LIB=<that .so>).  The snapshot
travels with gpurun like the main library.

  python tools/build_commit.py HEAD base            # HEAD's committed sources
  python tools/build_commit.py WORKTREE x -DFOO=1   # the working tree + flags
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = '/opt/rocm/bin/hipcc'
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off', '-fPIC', '-Wno-unused-result']
PARTS = (1, 3, 5, 7, 9, 11, 13, 15, 0)
SOURCES = ['include/gw_engine.h'] + [f'abmarl_amd/csrc/{f}' for f in
                                     ('gw_engine.hip', 'gw_lane.inc', 'gw_maze.inc', 'gw_pacman.inc', 'gw_rtt.inc')]


def main():
    commit, name, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = os.path.join(ROOT, 'abmarl_amd', '_build', 'ab', name)
    for rel in SOURCES:
        # the engine includes "../../include/gw_engine.h" from csrc/
        dst = os.path.join(out, rel) if rel.startswith('include') else os.path.join(out, 'src', rel.replace('abmarl_amd/', ''))
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        if commit == 'WORKTREE':
            with open(os.path.join(ROOT, rel)) as f:
                text = f.read()
        else:
            text = subprocess.check_output(['git', '-C', ROOT, 'show', f'{commit}:{rel}']).decode()
        with open(dst, 'w') as f:
            f.write(text)
    src = os.path.join(out, 'src', 'csrc', 'gw_engine.hip')
    jobs = [(os.path.join(out, 'host.o'), [])] + [(os.path.join(out, f'part_s{s}.o'), [f'-DGW_PART_S={s}'])
                                                  for s in PARTS]
    procs = [subprocess.Popen([HIPCC] + FLAGS + extra + x + ['-c', '-o', o, src]) for o, x in jobs]
    if any([p.wait() != 0 for p in procs]):   # wait for every job
        sys.exit(f'{name}: compile failed')
    lib = os.path.join(out, 'libgw_engine.so')
    subprocess.check_call([HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', lib] + [o for o, _ in jobs])
    print(lib)


if __name__ == '__main__':
    main()
