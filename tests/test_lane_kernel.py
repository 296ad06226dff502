"""The one-lane-per-env MazeNavigation kernel (abmarl_amd/csrc/gw_lane.inc)
against the C oracle and against the one-wave kernel, bit for bit.

Cases beyond BASELINE config 2 (test_engine_oracle.py): a small open maze
whose navigator starts next to the target (episodes of a few steps, so the
crowded-cell np.random.choice draw and the MT19937 twist at position 624 run
often, observer.py:236-246), observe_self off (no draw: the target's
encoding), env counts that are not a multiple of the 64 envs per wave, and
the reference's own examples/maze.txt layout."""
import numpy as np
import pytest

from tests.cases import load_golden, build_maze

pytestmark = pytest.mark.gpu

OPEN_MAZE = (
    'N_____',
    '_T__W_',
    '__W___',
    '_W____',
    '___W__',
    '______',
)


def _maze(maze, view_range=2, observe_self=True):
    cc = build_maze(dict(maze=[list(r) for r in maze], agent=dict(view_range=view_range))).compiled()
    cc.cfg.observe_self = int(observe_self)
    return cc


def _cases():
    return {
        'open': lambda: _maze(OPEN_MAZE),
        'open_no_self': lambda: _maze(OPEN_MAZE, observe_self=False),
        'open_view3': lambda: _maze(OPEN_MAZE, view_range=3),
        'maze_16': lambda: build_maze(load_golden('maze_16')['case']).compiled(),
        'maze_file': lambda: build_maze(load_golden('maze_file')['case']).compiled(),
    }


@pytest.mark.parametrize('name,E,horizon', [('open', 1000, 50), ('open_no_self', 777, 30),
                                            ('open_view3', 1024, 0), ('maze_file', 333, 80)])
def test_lane_kernel_vs_oracle(oracle_mod, name, E, horizon):
    from abmarl_amd import _abi
    from tests.test_engine_oracle import _run
    cc = _cases()[name]()
    _run(oracle_mod, cc, E=E, T=400, horizon=horizon, seed_run=9, key=17, kernel=_abi.GW_KERNEL_LANE)


def _engine(cc, E, env_per_lane, run):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc.cfg.env_per_lane = env_per_lane
    eng = GridWorldEngine(cc, E, seeds=env_seeds(E, run=run))
    eng.reset()
    eng.all_done.zero_()
    eng.set_state(steps=torch.as_tensor((np.arange(E) * 37 % 60).astype(np.int32), device=eng.device))
    return eng


@pytest.mark.parametrize('name', ['open', 'open_no_self', 'maze_16'])
@pytest.mark.parametrize('mode', ['next_step', 'same_step'])
def test_lane_kernel_vs_wave_kernel_rollout(name, mode):
    """gw_rollout fragments on both kernels (skip_done_obs on and off): every
    step's outputs, then the engine state and the MT19937 key + position."""
    import torch
    from abmarl_amd import _abi
    E = 640 + 17
    cc = _cases()[name]()
    a = _engine(cc, E, 0, run=3)
    b = _engine(cc, E, -1, run=3)
    assert a.kernel == _abi.GW_KERNEL_LANE and b.kernel == _abi.GW_KERNEL_WAVE
    t = 0
    for f, skip in ((40, False), (1, False), (57, True), (100, False)):
        acts = torch.empty((f,) + tuple(a.actions.shape), dtype=torch.int32, device=a.device)
        for s in range(f):
            a.random_actions(31, t + s, out=acts[s])
        oa = a.rollout(acts, horizon=60, autoreset=mode, skip_done_obs=skip)
        ob = b.rollout(acts, horizon=60, autoreset=mode, skip_done_obs=skip)
        for s in range(f):
            assert (oa['reward'][s].cpu().numpy().view(np.uint64) ==
                    ob['reward'][s].cpu().numpy().view(np.uint64)).all(), f"step {t + s}: reward"
            assert torch.equal(oa['done'][s], ob['done'][s]), f"step {t + s}: done"
            assert torch.equal(oa['all_done'][s], ob['all_done'][s]), f"step {t + s}: __all__"
            ga, gb = oa['obs'][s], ob['obs'][s]
            if skip:
                # rows without an observation are unwritten: compare the others
                live = (oa['done'][s] == 0) | (ob['done'][s] == 0)
                ga, gb = ga[live], gb[live]
            assert torch.equal(ga, gb), f"step {t + s}: obs"
        t += f
    sa, sb = a.get_state(), b.get_state()
    for k in ('pos', 'seq', 'health', 'steps'):
        assert torch.equal(sa[k], sb[k]), k
    assert torch.equal(sa['flags'] & 7, sb['flags'] & 7)
    ma = sa['mt'].cpu().numpy().view(np.uint32)
    mb = sb['mt'].cpu().numpy().view(np.uint32)
    assert (ma[:, :626] == mb[:, :626]).all(), "RNG key / position / seq counter"
    assert torch.equal(a.acting, b.acting)
    if cc.cfg.observe_self and name == 'open':
        assert (ma[:, 624] != 624).any(), "no draw happened: the case does not test the RNG path"


def test_lane_kernel_single_steps_and_explicit_resets():
    """The single-step C-ABI calls (gw_step, gw_step_autoreset) and explicit
    masked resets (the one-wave reset kernel) interleaved on one handle."""
    import torch
    cc = _cases()['open']()
    E = 200
    a = _engine(cc, E, 0, run=8)
    b = _engine(cc, E, -1, run=8)
    for t in range(120):
        act = a.random_actions(5, t)
        b.actions.copy_(act)
        if t % 3 == 0:
            ra = a.step(act)
            rb = b.step(b.actions)
        else:
            ra = a.step_autoreset(act, horizon=25)
            rb = b.step_autoreset(b.actions, horizon=25)
        for x, y in zip(ra, rb):
            assert torch.equal(x, y), f"step {t}"
        if t % 17 == 16:
            m = torch.as_tensor((np.arange(E) % 5 == t % 5).astype(np.uint8), device=a.device)
            assert torch.equal(a.reset(mask=m), b.reset(mask=m)), f"reset {t}"
            a.all_done.zero_(); b.all_done.zero_()
    sa, sb = a.get_state(), b.get_state()
    assert torch.equal(sa['pos'], sb['pos']) and torch.equal(sa['seq'], sb['seq'])
    ma = sa['mt'].cpu().numpy().view(np.uint32)
    mb = sb['mt'].cpu().numpy().view(np.uint32)
    assert (ma[:, :626] == mb[:, :626]).all()
