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


def test_struct_layout():
    # gw_agent_spec: 8 int32 + 3 double + int32 (+4 padding) = 64 bytes
    assert C.sizeof(_abi.AgentSpec) == 64
    assert _abi.Config.agents.offset % 8 == 0
    assert _abi.Config.pac_rewards.offset % 8 == 0


def test_create_rejects_bad_config_without_gpu(lib):
    # argument validation happens before any HIP call
    h = C.c_void_p()
    assert lib.gw_create(None, 4, 0, C.byref(h)) == _abi.GW_E_INVALID
    assert lib.gw_abi_version() == 3


def test_oracle_exports(oracle_mod):
    L = oracle_mod.lib()
    for f in ['gwo_create', 'gwo_seed', 'gwo_reset', 'gwo_step', 'gwo_get_state', 'gwo_destroy']:
        assert hasattr(L, f)
