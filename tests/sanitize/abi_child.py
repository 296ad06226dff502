"""Child process of tests/test_sanitizers.py::test_abi_validation_under_asan:
runs with the clang AddressSanitizer runtime preloaded and GW_ENGINE_LIB
pointing at the ASan + UBSan build of the host part.  Feeds gw_create the
malformed configurations it must reject (and valid ones, which get through the
whole validation and table building to the first HIP call), through ctypes.
Any sanitizer report aborts this process with a nonzero exit code."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from abmarl_amd import _abi, _native  # noqa: E402

maps = open('/proc/self/maps').read()
assert 'libclang_rt.asan' in maps, 'the ASan runtime is not loaded'
L = _native.lib()
assert os.path.basename(_native.variant_lib()) == 'libgw_engine_asan.so'
assert 'libgw_engine_asan.so' in open('/proc/self/maps').read()


def create(cc, n_envs=4):
    h = C.c_void_p()
    st = L.gw_create(C.cast(C.byref(cc.cfg), C.c_void_p), n_envs, 0, C.byref(h))
    if st == 0:
        L.gw_destroy(h)
    return st, L.gw_last_error().decode(errors='replace')


def team_battle_cc():
    from abmarl_amd.examples.workloads import team_battle_sim
    return team_battle_sim().compiled()


bad = []


def expect_reject(name, mutate, n_envs=4):
    cc = team_battle_cc()
    mutate(cc)
    st, msg = create(cc, n_envs)
    if st in (0, _abi.GW_E_HIP):
        bad.append((name, st, msg))


h = C.c_void_p()
assert L.gw_create(None, 4, 0, C.byref(h)) == _abi.GW_E_INVALID
expect_reject('zero envs', lambda cc: None, n_envs=0)
expect_reject('negative envs', lambda cc: None, n_envs=-3)
expect_reject('no agents', lambda cc: setattr(cc.cfg, 'n_agents', 0))
expect_reject('too many agents', lambda cc: setattr(cc.cfg, 'n_agents', 100000))
expect_reject('zero rows', lambda cc: setattr(cc.cfg, 'rows', 0))
expect_reject('negative cols', lambda cc: setattr(cc.cfg, 'cols', -5))
expect_reject('huge grid', lambda cc: (setattr(cc.cfg, 'rows', 4096), setattr(cc.cfg, 'cols', 4096)))
expect_reject('negative obs range', lambda cc: setattr(cc.cfg, 'obs_range', -1))
expect_reject('obs range too wide', lambda cc: setattr(cc.cfg, 'obs_range', 1000))
expect_reject('unknown program', lambda cc: setattr(cc.cfg, 'sim_kind', 77))
for field, value in (('encoding', 0), ('encoding', _abi.GW_MAX_ENC + 1), ('init_row', 10 ** 6),
                     ('init_col', 10 ** 6), ('view_range', 10 ** 6), ('attack_range', 10 ** 6),
                     ('move_range', -7), ('simultaneous_attacks', -1), ('attack_strength', 1.5),
                     ('attack_accuracy', float('nan')), ('initial_health', 3.0)):
    def mut(cc, field=field, value=value):
        setattr(cc.cfg.agents[3], field, value)
    expect_reject(f'agent {field}={value}', mut)
expect_reject('pacman without its agent', lambda cc: (setattr(cc.cfg, 'sim_kind', _abi.GW_SIM_PACMAN),
                                                       setattr(cc.cfg, 'pacman_agent', -1)))
# valid configurations: the whole validation and host-side table building,
# then hipSetDevice / hipMalloc, which fail without a GPU (GW_E_HIP)
from abmarl_amd.examples.workloads import maze_sim, rtt_sim, pacman_sim  # noqa: E402
for build in (team_battle_cc, lambda: maze_sim().compiled(), lambda: rtt_sim().compiled(),
              lambda: pacman_sim().compiled()):
    st, msg = create(build())
    assert st in (0, _abi.GW_E_HIP), (st, msg)
assert not bad, bad
print('abi validation under ASan: ok')
