"""Replay a golden fixture through a runner and compare bit-exactly."""
import zlib

import numpy as np


def _bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)


def check_step(g, t, obs, rew, done, all_done, state=None, where='', errors=None):
    """Compare one step.  Envs whose reference step raised (fixture 'err':
    ReachTheTarget's double remove) have no reference outputs: for them only
    the error flag and the RNG state are checked."""
    E = g['all_done'].shape[1]
    code = g['err'][t] if 'err' in g else np.zeros(E, np.uint8)
    err = code != 0
    if err.any():
        # the fixture's exception (1 KeyError, 2 ValueError) -> the engine's flag
        assert errors is not None, f"{where} step {t}: runner reports no errors"
        for c, flag, name in ((1, 4, 'KeyError'), (2, 32, 'ValueError')):
            assert ((errors[code == c] & flag) != 0).all(), f"{where} step {t}: {name} flag missing"
            assert ((errors[code != c] & flag) == 0).all(), f"{where} step {t}: spurious {name} flag"
        g = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in g.items()}
        g['obs'][t][err] = obs[err]
        g['reward'][t][err] = rew[err]
        g['done'][t][err] = done[err]
        g['all_done'][t][err] = all_done[err]
        if state is not None:
            g['pos'][t][err] = state['pos'][err]
            g['health'][t][err] = state['health'][err]
            g['active'][t][err] = ((state['flags'] >> 2) & 1)[err]
            if 'ammo' in g and 'ammo' in state:
                g['ammo'][t][err] = state['ammo'][err]
    ok_obs = obs.astype(np.int64) == g['obs'][t].astype(np.int64)
    assert ok_obs.all(), f"{where} step {t}: obs mismatch at {np.argwhere(~ok_obs)[:5].tolist()}"
    bad = _bits(rew) != _bits(g['reward'][t])
    assert not bad.any(), (f"{where} step {t}: reward mismatch at {np.argwhere(bad)[:5].tolist()}: "
                           f"{rew[bad][:5]} vs {g['reward'][t][bad][:5]}")
    assert (done == g['done'][t]).all(), f"{where} step {t}: done mismatch"
    assert (all_done == g['all_done'][t]).all(), f"{where} step {t}: __all__ mismatch"
    if state is not None:
        assert (state['pos'] == g['pos'][t]).all(), f"{where} step {t}: positions differ"
        h = state['health']
        assert (h == g['health'][t]).all(), f"{where} step {t}: health differs"
        act = (state['flags'] >> 2) & 1
        assert (act == g['active'][t]).all(), f"{where} step {t}: active differs"
        if 'ammo' in g and 'ammo' in state:
            assert (state['ammo'] == g['ammo'][t]).all(), f"{where} step {t}: ammo differs"
        mt = state['mt']
        for e in range(E):
            assert int(mt[e, 624]) == int(g['mt_pos'][t, e]), f"{where} step {t} env {e}: RNG pos"
            crc = zlib.crc32(np.ascontiguousarray(mt[e, :624], dtype=np.uint32).tobytes())
            assert crc == int(g['mt_crc'][t, e]), f"{where} step {t} env {e}: RNG key digest"


def replay(runner, g, with_state=True, steps=None):
    """runner API: reset(mask=None) -> obs (E,A,S,S); step(actions) -> (obs, rew, done, all_done);
    state() -> dict(pos, health, flags, mt)."""
    obs0 = runner.reset(None)
    assert (obs0 == g['obs0']).all(), "initial reset obs mismatch"
    T = g['actions'].shape[0] if steps is None else steps
    for t in range(T):
        obs, rew, done, all_done = runner.step(g['actions'][t].astype(np.int32))
        st = runner.state() if with_state else None
        errs = runner.errors() if hasattr(runner, 'errors') else None
        check_step(g, t, obs, rew, done, all_done, st, where=type(runner).__name__, errors=errs)
        m = g['reset_mask'][t].astype(np.uint8)
        if m.any():
            robs = runner.reset(m)
            sel = m.astype(bool)
            assert (robs[sel] == g['reset_obs'][t][sel]).all(), f"step {t}: reset obs mismatch"
    return T
