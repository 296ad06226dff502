"""CPU sanitizer runs (`-fsanitize=address` on the CPU build).

  * the C oracle built with AddressSanitizer + UBSan (oracle/Makefile
    build/asan/, every UB report fatal) replays the reference's golden
    trajectories and the Maze / Pacman oracle tests in a child process that
    preloads libasan;
  * the host half of the C-ABI (gw_engine.hip's host part: gw_create's
    config validation and host-side table building) built with
    `-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined`, the
    per-window-side kernel parts replaced by stubs (tests/sanitize/
    part_stubs.cpp), is fed the malformed configurations gw_create must
    reject and the BASELINE programs' valid ones (tests/sanitize/
    abi_child.py) under the clang ASan runtime.

A sanitizer report aborts the child, so the test fails on any finding.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG_ASAN = '/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so'
ABI_LIB = os.path.join(ROOT, 'abmarl_amd', '_build', 'libgw_engine_asan.so')


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ('GW_ENGINE_LIB', 'GW_ENGINE_VARIANT')}
    e.update(ASAN_OPTIONS='detect_leaks=0:abort_on_error=1', UBSAN_OPTIONS='halt_on_error=1:print_stacktrace=1',
             OMP_NUM_THREADS='2', PYTHONDONTWRITEBYTECODE='1')
    e.update(kw)
    return e


def test_oracle_golden_replays_under_asan_ubsan():
    libasan = subprocess.check_output(['gcc', '-print-file-name=libasan.so'], text=True).strip()
    if not os.path.isabs(libasan):
        pytest.skip('gcc has no libasan')
    env = _env(GW_ORACLE_SANITIZE='1', LD_PRELOAD=libasan)
    # the instrumented library really is the one loaded
    probe = ("from oracle import oracle; L = oracle.lib(); import os; "
             "m = open('/proc/self/maps').read(); "
             "assert 'build/asan/libgw_oracle.so' in m and 'libasan' in m, 'not the ASan oracle'")
    subprocess.run([sys.executable, '-c', probe], cwd=ROOT, env=env, check=True, timeout=600)
    r = subprocess.run([sys.executable, '-m', 'pytest', '-x', '-q', '-p', 'no:cacheprovider', '-m', 'not gpu',
                        'tests/test_oracle_golden.py', 'tests/test_maze_oracle.py', 'tests/test_pacman_oracle.py'],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert 'passed' in r.stdout


def build_abi_asan():
    """libgw_engine_asan.so: the host part with ASan + UBSan on the host side
    linked with the part stubs (the host part's own kernels are compiled
    as usual; only the host side is instrumented)."""
    from abmarl_amd import _native
    srcs = [_native.SRC, _native.INCLUDE, os.path.join(ROOT, 'tests', 'sanitize', 'part_stubs.cpp')]
    if os.path.exists(ABI_LIB) and os.path.getmtime(ABI_LIB) >= max(os.path.getmtime(s) for s in srcs):
        return ABI_LIB
    objdir = os.path.join(ROOT, 'abmarl_amd', '_build', 'obj_asan')
    os.makedirs(objdir, exist_ok=True)
    san = ['-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fsanitize=undefined',
           '-Xarch_host', '-fno-sanitize-recover=all', '-Xarch_host', '-fno-omit-frame-pointer']
    host_o = os.path.join(objdir, 'host.o')
    stub_o = os.path.join(objdir, 'stubs.o')
    subprocess.check_call([_native.HIPCC, '--offload-arch=gfx950', '-O1', '-g',
                           '-std=c++17', '-fPIC', '-Wno-unused-result'] + san +
                          ['-c', '-o', host_o, _native.SRC])
    subprocess.check_call([_native.HIPCC, '-O1', '-std=c++17', '-fPIC', '-c', '-o', stub_o, srcs[2]])
    subprocess.check_call([_native.HIPCC, '-shared', '-fPIC', '-fsanitize=address,undefined',
                           '-o', ABI_LIB + '.tmp', host_o, stub_o])
    os.replace(ABI_LIB + '.tmp', ABI_LIB)
    return ABI_LIB


def test_abi_validation_under_asan():
    if not os.path.exists(CLANG_ASAN):
        pytest.skip('no clang ASan runtime')
    lib = build_abi_asan()
    env = _env(GW_ENGINE_LIB=lib, LD_PRELOAD=CLANG_ASAN, HIP_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'sanitize', 'abi_child.py')],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert 'abi validation under ASan: ok' in r.stdout
