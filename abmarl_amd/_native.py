"""Loader for the HIP engine library (libgw_engine.so, built in-tree).

The product path has no CPU fallback: if the library or a GPU is missing,
``lib()`` raises.
"""
import ctypes as C
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(PKG, 'csrc', 'gw_engine.hip')
INCLUDE = os.path.join(os.path.dirname(PKG), 'include', 'gw_engine.h')
LIB = os.path.join(PKG, '_build', 'libgw_engine.so')
# A/B runs of another in-tree build (tools/ab_*.py); never set by the product path
if os.environ.get('GW_ENGINE_LIB'):
    LIB = os.path.abspath(os.environ['GW_ENGINE_LIB'])
# diagnostic build with in-kernel s_memtime stamps (tools/stamps.py); never the default
LIB_STAMPS = os.path.join(PKG, '_build', 'libgw_engine_stamps.so')
# diagnostic build with bounds / one-lane checks that record instead of faulting
LIB_CHECKS = os.path.join(PKG, '_build', 'libgw_engine_checks.so')
VARIANT = os.environ.get('GW_ENGINE_VARIANT', '')   # '', 'stamps' or 'checks'
if os.environ.get('GW_ENGINE_STAMPS') == '1':
    VARIANT = 'stamps'


def variant_lib(variant=None):
    v = VARIANT if variant is None else variant
    # GW_ENGINE_LIB (diagnostic runs only) replaces the selected variant's library
    if variant is None and os.environ.get('GW_ENGINE_LIB'):
        return LIB
    return {'': LIB, 'stamps': LIB_STAMPS, 'checks': LIB_CHECKS}[v]
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('GW_OFFLOAD_ARCH', 'gfx950')

# every entry point declared in include/gw_engine.h: (restype, argtypes)
_vp, _i32, _u32, _u64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64
SIGNATURES = {
    'gw_create': (_i32, [_vp, _i32, _i32, C.POINTER(_vp)]),
    'gw_seed': (_i32, [_vp, _vp, _vp]),
    'gw_reset': (_i32, [_vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    'gw_step': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'gw_step_autoreset': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    'gw_step_autoreset_next': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    'gw_get_state': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'gw_set_state': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'gw_random_actions': (_i32, [_vp, _u64, _u32, _u32, _vp, _vp]),
    'gw_rollout_step': (_i32, [_vp, _u64, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32,
                               _vp, _vp]),
    'gw_rollout': (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    'gw_set_launch_events': (_i32, [_vp, _vp, _vp]),
    'gw_component': (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    'gw_generate_maze': (_i32, [_vp, _vp, _vp, _vp]),
    'gw_destroy': (_i32, [_vp]),
    'gw_num_envs': (_i32, [_vp]),
    'gw_obs_side': (_i32, [_vp]),
    'gw_num_lanes': (_i32, [_vp]),
    'gw_env_kernel': (_i32, [_vp]),
    'gw_act_dim': (_i32, [_vp]),
    'gw_step_occupancy': (_i32, [_vp, _vp, _vp, _vp]),
    'gw_set_placement_order': (_i32, [_vp, _vp, _i32]),
    'gw_set_action_order': (_i32, [_vp, _vp, _i32]),
    'gw_lane_entities': (_i32, [_vp, _vp]),
    'gw_obs_shape': (_i32, [_vp, _vp, _vp]),
    'gw_num_passive': (_i32, [_vp]),
    'gw_turn_reset': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'gw_turn_step': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    'gw_turn_rollout': (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    'gw_sim_reset': (_i32, [_vp, _vp, _vp, _vp]),
    'gw_sim_step': (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'gw_observe': (_i32, [_vp, _i32, _vp, _vp]),
    'gw_get_aux_state': (_i32, [_vp, _vp, _vp, _vp, _vp]),
    'gw_get_ammo': (_i32, [_vp, _vp, _vp]),
    'gw_set_ammo': (_i32, [_vp, _vp, _vp]),
    'gw_set_aux_state': (_i32, [_vp, _vp, _vp, _vp, _vp]),
    'gw_last_error': (C.c_char_p, []),
    'gw_abi_version': (_i32, []),
}


PART_SIDES = (1, 3, 5, 7, 9, 11, 13, 15, 0)   # observation window sides S = 2*range+1; 0: any S > 15


def build(force=False, verbose=False, stamps=False, checks=False, out=None, extra_flags=()):
    """Compile the engine for gfx950 with hipcc (works without a GPU).

    gw_engine.hip is compiled as one host part plus one part per window side
    S (-DGW_PART_S, the templated step/reset kernels), in parallel, then
    linked into one shared library."""
    out = out or (LIB_STAMPS if stamps else (LIB_CHECKS if checks else LIB))
    csrc = os.path.dirname(SRC)
    deps = [SRC, INCLUDE] + [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith('.inc')]
    if not force and os.path.exists(out) and \
            os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tag = 'stamps' if stamps else ('checks' if checks else 'prod')
    if extra_flags:   # tools' A/B builds (tools/ab_lib.py)
        tag = os.path.splitext(os.path.basename(out))[0]
    flags = [f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-ffp-contract=off', '-fPIC',
             '-Wno-unused-result'] + (['-DGW_STAMPS'] if stamps else []) + \
        (['-DGW_CHECKS'] if checks else []) + list(extra_flags)
    objdir = os.path.join(os.path.dirname(out), f'obj_{tag}')
    os.makedirs(objdir, exist_ok=True)
    jobs = [(os.path.join(objdir, 'host.o'), [])] + \
        [(os.path.join(objdir, f'part_s{s}.o'), [f'-DGW_PART_S={s}']) for s in PART_SIDES]
    cmds = [[HIPCC] + flags + extra + ['-c', '-o', o, SRC] for o, extra in jobs]
    if verbose:
        for c in cmds:
            print(' '.join(c))
    par = max(1, min(len(cmds), int(os.environ.get('MAX_JOBS', '0')) or (os.cpu_count() or 1)))
    running, failed = [], []
    pending = list(cmds)
    while pending or running:
        while pending and len(running) < par:
            c = pending.pop(0)
            running.append((c, subprocess.Popen(c)))
        c, pr = running.pop(0)
        if pr.wait() != 0:
            failed.append(' '.join(c))
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', out + '.tmp'] + [o for o, _ in jobs]
    if verbose:
        print(' '.join(link))
    subprocess.check_call(link)
    os.replace(out + '.tmp', out)
    return out


_lib = None


def lib():
    """The loaded engine library; raises if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(variant_lib()):
            raise RuntimeError(f"HIP engine library {LIB} is missing; run "
                               "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(variant_lib())
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class EngineError(RuntimeError):
    pass


def check(status, what):
    if status != 0:
        msg = lib().gw_last_error().decode(errors='replace')
        raise EngineError(f"{what} failed with status {status}: {msg}")
