"""gw_rollout (one launch for a fragment of K steps) against K single-step
calls on an engine with the same seeds, bit for bit: every step's obs,
float64 reward bits, dones and __all__, and the final engine state
(positions, health, flags, RNG, step counters, acting counters).  The
single-step calls are themselves pinned to the reference fixtures and the
oracle (test_engine_golden.py, test_engine_oracle.py)."""
import numpy as np
import pytest

from tests.cases import team_battle, load_golden, build_maze, build_rtt, RTT_CONFIG4

pytestmark = pytest.mark.gpu


def _pair(cc, E, run=0, stagger=0, force_workgroup=False):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc.cfg.force_workgroup = int(force_workgroup)
    engs = [GridWorldEngine(cc, E, seeds=env_seeds(E, run=run)) for _ in range(2)]
    for eng in engs:
        eng.reset()
        eng.all_done.zero_()
        if stagger:
            eng.set_state(steps=torch.as_tensor((np.arange(E) * stagger // E).astype(np.int32),
                                                device=eng.device))
    return engs


def _actions(eng, key, t0, K):
    import torch
    acts = torch.empty((K,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
    for t in range(K):
        eng.random_actions(key, t0 + t, out=acts[t])
    return acts


def _compare(ra, rb, K, horizon, mode, key=5, frags=(1, 7, 16), skip=False, allow_err=False):
    """Engine a: fragments of the given sizes through gw_rollout; engine b: the
    same steps one call at a time."""
    step_b = rb.step_autoreset_next if mode == 'next_step' else rb.step_autoreset
    t = 0
    err_b = rb.err.cpu().numpy().copy()
    for f in frags:
        acts = _actions(ra, key, t, f)
        out = ra.rollout(acts, horizon=horizon, autoreset=mode, skip_done_obs=skip)
        for s in range(f):
            rb.err.zero_()
            obs, rew, done, ad = step_b(acts[s].contiguous(), horizon=horizon)
            # an env whose step raised (ReachTheTarget's double remove) has
            # that step's reward / done (and, NEXT_STEP, obs) unwritten
            raised = rb.err.cpu().numpy() != 0
            err_b |= rb.err.cpu().numpy()
            ok = ~raised
            rw = out['reward'][s].cpu().numpy().view(np.uint64)
            assert (rw[ok] == rew.cpu().numpy().view(np.uint64)[ok]).all(), f"step {t + s}: reward"
            assert (out['done'][s].cpu().numpy()[ok] == done.cpu().numpy()[ok]).all(), f"step {t + s}: done"
            assert (out['all_done'][s].cpu().numpy() == ad.cpu().numpy()).all(), f"step {t + s}: __all__"
            go, bo = out['obs'][s].cpu().numpy(), obs.cpu().numpy()
            if mode == 'next_step':
                go, bo = go[ok], bo[ok]
            if skip:
                # rows of lanes without an observation this step are unspecified
                m = (bo != -2).reshape(bo.shape[0], bo.shape[1], -1).any(-1)
                assert (go[m] == bo[m]).all(), f"step {t + s}: obs"
            else:
                assert (go == bo).all(), f"step {t + s}: obs"
        t += f
    sa, sb = ra.get_state(), rb.get_state()
    for k in ('pos', 'health', 'seq', 'steps'):
        assert (sa[k].cpu().numpy() == sb[k].cpu().numpy()).all(), k
    assert ((sa['flags'].cpu().numpy() & 7) == (sb['flags'].cpu().numpy() & 7)).all(), 'flags'
    mt_a, mt_b = sa['mt'].cpu().numpy(), sb['mt'].cpu().numpy()
    assert (mt_a[:, :625] == mt_b[:, :625]).all(), 'RNG'
    assert (ra.acting.cpu().numpy() == rb.acting.cpu().numpy()).all(), 'acting'
    if not allow_err:
        assert not ra.err.any().item()
    assert (ra.err.cpu().numpy() == err_b).all(), 'err flags'
    rb.err.copy_(ra.err)


@pytest.mark.parametrize('mode', ['next_step', 'same_step'])
def test_rollout_team_battle_headline(mode):
    """The headline config (32x32, 64 agents) at 1024 envs, start phases
    staggered over a short horizon so that resets land inside fragments."""
    a, b = _pair(team_battle(), 1024, run=2, stagger=30)
    _compare(a, b, 24, horizon=30, mode=mode, frags=(1, 7, 16, 40))


def test_rollout_skip_done_obs():
    """skip_done_obs: every written row is the single-step call's."""
    a, b = _pair(team_battle(), 512, run=3, stagger=25)
    _compare(a, b, 0, horizon=25, mode='next_step', frags=(20, 20), skip=True)


def test_rollout_headline_full_size_bench_shape():
    """The headline bench's launch shape: 4096 envs, episodes staggered over
    the 200-step horizon (a reset lands in every step), 20-step fragments,
    skip_done_obs, next-step auto-reset (bench.py run_rollout)."""
    a, b = _pair(team_battle(), 4096, run=1, stagger=200)
    _compare(a, b, 0, horizon=200, mode='next_step', frags=(20, 20), skip=True)


def test_rollout_workgroup_kernel_8192_envs():
    """Config 4's 8192-envs-on-one-GPU launch shape (bench.py
    other_configs.reach_the_target_64_all_8192) as one 30-step fragment
    against single steps."""
    kw = {k: v for k, v in RTT_CONFIG4.items() if k != 'kind'}
    cc = build_rtt(dict(kind='rtt', **kw)).compiled()
    a, b = _pair(cc, 8192, run=8, stagger=20)
    assert a.wg
    _compare(a, b, 0, horizon=20, mode='next_step', frags=(30,), skip=True, allow_err=True)


def test_restored_snapshot_rewrites_done_rows():
    """A snapshot restored into another engine (gw_get_state -> reset ->
    gw_set_state): the next step writes every row, so done entities show -2
    again (the engine-internal obs-row bit does not travel with a snapshot)."""
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc = team_battle(rows=8, cols=8, n_agents=40, n_teams=2,
                     agent=dict(move_range=1, attack_range=1, attack_strength=1,
                                attack_accuracy=1, view_range=2))
    E = 256
    a = GridWorldEngine(cc, E, seeds=env_seeds(E, run=9))
    b = GridWorldEngine(cc, E, seeds=env_seeds(E, run=10))
    a.reset()
    for t in range(12):
        a.step(a.random_actions(3, t))
    assert a.done.any().item(), "some entity is done by now"
    snap = a.get_state()
    assert not (snap['flags'] & 0x40).any().item(), "snapshot carries the internal bit"
    b.reset()
    b.set_state(**snap)
    # entities done BEFORE this step get no observation (-2); one that dies
    # in it is still observed (all_step_manager.py:68-79)
    dead = a.done.cpu().numpy().astype(bool)
    act = a.random_actions(3, 12)
    oa = a.step(act)[0].cpu().numpy()
    ob = b.step(act)[0].cpu().numpy()
    assert (oa == ob).all()
    assert dead.any() and (ob[dead] == -2).all()
    torch.cuda.synchronize()


def test_rollout_dense_small_grid():
    """Crowded 8x8 grid, 40 agents in 3 teams (crowded-cell draws, kills,
    one-team-remaining ends inside fragments)."""
    cc = team_battle(rows=8, cols=8, n_agents=40, n_teams=3,
                     agent=dict(move_range=1, attack_range=1, attack_strength=0.5,
                                attack_accuracy=0.7, view_range=2))
    a, b = _pair(cc, 512, run=4)
    _compare(a, b, 0, horizon=50, mode='next_step', frags=(33, 33, 1))


def test_rollout_maze():
    cc = build_maze(load_golden('maze_16')['case']).compiled()
    a, b = _pair(cc, 256, run=5, stagger=40)
    _compare(a, b, 0, horizon=40, mode='next_step', frags=(30, 30))


def test_rollout_reach_the_target_double_remove():
    """ReachTheTarget on the one-wave kernel, crowded enough that the
    double remove (KeyError) fires inside fragments."""
    from tests.test_engine_oracle import RTT_WAVE_CASES
    cc = build_rtt(dict(kind='rtt', **RTT_WAVE_CASES[1])).compiled()
    a, b = _pair(cc, 256, run=6)
    _compare(a, b, 0, horizon=40, mode='next_step', frags=(25, 25), allow_err=True)
    _compare(a, b, 0, horizon=40, mode='same_step', frags=(25,), allow_err=True)


def test_rollout_workgroup_kernel():
    """The workgroup-per-env kernel (BASELINE config 4 at 64 envs): the
    fragment runs in one launch (each env's state passes through HBM between
    its steps), same results as single steps, both auto-reset modes."""
    kw = {k: v for k, v in RTT_CONFIG4.items() if k != 'kind'}
    cc = build_rtt(dict(kind='rtt', **kw)).compiled()
    a, b = _pair(cc, 64, run=7, stagger=20)
    assert a.wg
    _compare(a, b, 0, horizon=20, mode='next_step', frags=(12, 1, 30), allow_err=True)
    _compare(a, b, 0, horizon=20, mode='same_step', frags=(25,), allow_err=True)


def test_rollout_workgroup_kernel_double_remove():
    """The crowded ReachTheTarget case forced through the workgroup kernel:
    the double remove (KeyError) fires inside fragments."""
    from tests.test_engine_oracle import RTT_WAVE_CASES
    cc = build_rtt(dict(kind='rtt', **RTT_WAVE_CASES[1])).compiled()
    a, b = _pair(cc, 256, run=6, force_workgroup=True)
    assert a.wg
    _compare(a, b, 0, horizon=40, mode='next_step', frags=(25, 25), allow_err=True)
    _compare(a, b, 0, horizon=40, mode='same_step', frags=(25,), allow_err=True)


def test_rollout_workgroup_team_battle():
    """TeamBattle with 128 fighters (the workgroup kernel) as fragments."""
    cc = team_battle(rows=32, cols=32, n_agents=128, n_teams=2)
    a, b = _pair(cc, 256, run=9, stagger=30)
    assert a.wg
    _compare(a, b, 0, horizon=30, mode='next_step', frags=(20, 20))
    _compare(a, b, 0, horizon=30, mode='same_step', frags=(15,))


@pytest.mark.parametrize('waves', [2, 4])
def test_rollout_multi_wave_team_battle(waves):
    """The headline TeamBattle config on the workgroup kernel with 2 / 4
    waves per env (the small-batch variant) as fragments vs single steps."""
    cc = team_battle()
    a, b = _pair(cc, 256, run=10, stagger=30, force_workgroup=waves)
    assert a.wg
    _compare(a, b, 0, horizon=30, mode='next_step', frags=(20, 20), skip=True)
    _compare(a, b, 0, horizon=30, mode='same_step', frags=(15,))


def test_rollout_multi_wave_double_remove():
    """A crowded ReachTheTarget case (fewer than 64 lanes) on 4 waves."""
    from tests.test_engine_oracle import RTT_WAVE_CASES
    cc = build_rtt(dict(kind='rtt', **RTT_WAVE_CASES[1])).compiled()
    a, b = _pair(cc, 256, run=6, force_workgroup=4)
    assert a.wg
    _compare(a, b, 0, horizon=40, mode='next_step', frags=(25, 25), allow_err=True)


def test_rollout_traffic_corridor():
    from tests.cases import build_traffic
    cc = build_traffic(load_golden('traffic_9')['case']).compiled()
    a, b = _pair(cc, 256, run=8, stagger=30)
    _compare(a, b, 0, horizon=30, mode='next_step', frags=(40, 40))
