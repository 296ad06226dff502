"""The C-ABI library loads (no GPU needed) and exports every entry point
declared in include/gw_engine.h; the ctypes mirror matches the header."""
import ctypes as C
import os
import re

import pytest

from abmarl_amd import _abi, _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'gw_engine.h')


def header_functions():
    """Exported entry points (header-only `static inline` helpers excluded)."""
    txt = open(HEADER).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    inline = set(re.findall(r'static\s+inline\s+\w+\s+(gw_[a-z_]+)\s*\(', txt))
    txt = re.sub(r'static\s+inline[^{]*\{.*?\n\}', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(gw_[a-z_]+)\s*\(', txt)) - inline)


def header_defines():
    out = {}
    for m in re.finditer(r'#define\s+(GW_[A-Z0-9_]+)\s+\(?(-?[0-9xa-fA-F]+)u?\)?', open(HEADER).read()):
        out[m.group(1)] = int(m.group(2).rstrip('u'), 0)
    return out


@pytest.fixture(scope='module')
def lib():
    _native.build()
    return _native.lib()


def test_every_declared_symbol_is_exported(lib):
    fns = header_functions()
    assert len(fns) >= 12
    for f in fns:
        assert hasattr(lib, f), f"{f} declared in include/gw_engine.h but not exported"
        assert f in _native.SIGNATURES, f"{f} missing from the ctypes signature table"


def test_constants_match_header():
    for name, val in header_defines().items():
        if hasattr(_abi, name):
            assert getattr(_abi, name) == val, name


def test_struct_layout(tmp_path):
    """The ctypes mirror of gw_agent_spec / gw_config has the C compiler's
    size and field offsets (a tiny C program compiled against the header)."""
    import subprocess
    fields = {'gw_agent_spec': [f for f, _ in _abi.AgentSpec._fields_],
              'gw_config': [f for f, _ in _abi.Config._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', 'int main(void) {']
    for st, fs in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines += ['return 0; }']
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'layout'
    subprocess.check_call(['gcc', '-o', str(exe), str(src)])
    got = dict(line.rsplit(' ', 1) for line in subprocess.check_output([str(exe)]).decode().split('\n') if line)
    py = {'gw_agent_spec': _abi.AgentSpec, 'gw_config': _abi.Config}
    for st, cls in py.items():
        assert int(got[st]) == C.sizeof(cls), st
        for f in fields[st]:
            assert int(got[f'{st}.{f}']) == getattr(cls, f).offset, f'{st}.{f}'


def test_create_rejects_bad_config_without_gpu(lib):
    # argument validation happens before any HIP call
    h = C.c_void_p()
    assert lib.gw_create(None, 4, 0, C.byref(h)) == _abi.GW_E_INVALID
    assert lib.gw_abi_version() == 7


def test_oracle_exports(oracle_mod):
    L = oracle_mod.lib()
    for f in ['gwo_create', 'gwo_seed', 'gwo_reset', 'gwo_step', 'gwo_get_state', 'gwo_destroy']:
        assert hasattr(L, f)
