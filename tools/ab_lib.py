"""Build an A/B variant of the engine library quickly: only the window-side
part(s) named are recompiled with the extra flags, the rest is linked from
the production build's objects (abmarl_amd/_build/obj_prod, so run the
production build first).

  python tools/ab_lib.py <name> <S|host>[,<S|host>...] [-DFLAG ...]
(recompile the host part too when a flag changes host-side launch geometry)
  -> abmarl_amd/_build/libgw_engine_<name>.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from abmarl_amd import _native  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[3:]
    parts = sys.argv[2].split(',')
    host = 'host' in parts
    sides = [int(s) for s in parts if s != 'host']
    bdir = os.path.dirname(_native.LIB)
    prod = os.path.join(bdir, 'obj_prod')
    odir = os.path.join(bdir, f'obj_ab_{name}')
    os.makedirs(odir, exist_ok=True)
    base = [f'--offload-arch={_native.ARCH}', '-O3', '-std=c++17', '-ffp-contract=off', '-fPIC',
            '-Wno-unused-result', '-Wno-pass-failed']
    procs = []
    for s in sides:
        o = os.path.join(odir, f'part_s{s}.o')
        procs.append(subprocess.Popen([_native.HIPCC] + base + flags + [f'-DGW_PART_S={s}', '-c', '-o', o,
                                                                        _native.SRC]))
    if host:
        procs.append(subprocess.Popen([_native.HIPCC] + base + flags + ['-c', '-o', os.path.join(odir, 'host.o'),
                                                                        _native.SRC]))
    if any(p.wait() != 0 for p in procs):
        raise SystemExit('compile failed')
    objs = [os.path.join(odir if host else prod, 'host.o')] + \
        [os.path.join(odir if s in sides else prod, f'part_s{s}.o') for s in _native.PART_SIDES]
    out = os.path.join(bdir, f'libgw_engine_{name}.so')
    subprocess.check_call([_native.HIPCC, f'--offload-arch={_native.ARCH}', '-shared', '-fPIC', '-o', out] + objs)
    print(out)


if __name__ == '__main__':
    main()
