"""HIP engine vs the C oracle at scale: the headline TeamBattle configuration
(32x32, 64 agents, 2 teams) with random-policy actions, in-launch auto-reset,
compared bit-exactly every step (obs, float64 reward bits, dones, __all__)
and on the final engine state (positions, health, flags, RNG)."""
import numpy as np
import pytest

from tests.cases import team_battle, load_golden, build_maze

pytestmark = pytest.mark.gpu


def _run(oracle_mod, cc, E, T, horizon, seed_run, key, check_every=1, force_workgroup=False,
         env_per_lane=0, kernel=None, as_list=False):
    """The oracle holds every entity, the engine one lane per dynamic entity:
    compare the lanes (static entities are constant in both).  as_list: the
    attacked agents read as a list (gw_config.attack_array_as_list) -- configs
    attacking 2-3 times a step, whose reference step would raise ValueError
    (that path: test_team_battle_value_error)."""
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    seeds = env_seeds(E, run=seed_run)
    cc.cfg.force_workgroup = int(force_workgroup)
    cc.cfg.attack_array_as_list = int(as_list)
    cc.cfg.env_per_lane = int(env_per_lane)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    assert eng.wg == (bool(force_workgroup) or eng.A > 64)
    if kernel is not None:
        assert eng.kernel == kernel, (eng.kernel, kernel)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    NE, ln = cc.n_agents, eng.lane_entities
    o_obs = orc.new_obs()
    orc.reset(o_obs)
    g_obs = eng.reset().cpu().numpy()
    assert (g_obs == o_obs[:, ln]).all(), "reset obs"
    rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8); ad = np.zeros(E, np.uint8)
    h_act = np.zeros((E, NE, 3), np.int32)
    for t in range(T):
        act = eng.random_actions(key, t)
        h_act[:, ln] = act.cpu().numpy()
        orc.step(h_act, o_obs, rew, done, ad)
        orc.reset(o_obs, all_done=ad, horizon=horizon)
        obs, r, d, a = eng.step_autoreset(act, horizon=horizon)
        assert (r.cpu().numpy().view(np.uint64) == rew[:, ln].view(np.uint64)).all(), f"step {t}: reward"
        assert (d.cpu().numpy() == done[:, ln]).all(), f"step {t}: done"
        assert (a.cpu().numpy() == ad).all(), f"step {t}: __all__"
        if t % check_every == 0 or t == T - 1:
            g = obs.cpu().numpy()
            bad = g != o_obs[:, ln]
            assert not bad.any(), f"step {t}: obs mismatch at {np.argwhere(bad)[:3].tolist()}"
    torch.cuda.synchronize()
    st = eng.get_state()
    ost = orc.state()
    assert (st['pos'].cpu().numpy() == ost['pos'][:, ln]).all()
    assert (st['health'].cpu().numpy() == ost['health'][:, ln]).all()
    assert (st['flags'].cpu().numpy() & 7 == ost['flags'][:, ln]).all()
    mt = st['mt'].cpu().numpy().view(np.uint32)
    assert (mt[:, :625] == ost['mt'][:, :625]).all(), "RNG state"
    assert not eng.err.any().item()


def test_headline_config_4096_envs(oracle_mod):
    cc = team_battle()
    _run(oracle_mod, cc, E=4096, T=160, horizon=70, seed_run=0, key=11, check_every=4)


@pytest.mark.parametrize('kw', [
    # accuracy < 1, crowded, 3 teams
    dict(rows=8, cols=8, n_agents=40, n_teams=3,
         agent=dict(move_range=1, attack_range=1, attack_strength=1, attack_accuracy=0.6, view_range=2)),
    # attack range 2: up to 25 window cells
    dict(rows=10, cols=10, n_agents=48, n_teams=2,
         agent=dict(move_range=1, attack_range=2, attack_strength=1, attack_accuracy=0.9, view_range=3)),
])
def test_dense_attack_configs(oracle_mod, kw):
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=1024, T=100, horizon=40, seed_run=8, key=21, check_every=2)


@pytest.mark.parametrize('kw', [
    dict(rows=8, cols=8, n_agents=16, n_teams=2),
    dict(rows=5, cols=5, n_agents=20, n_teams=4),
    dict(rows=12, cols=20, n_agents=64, n_teams=3,
         overlap={'1': [1, 2], '2': [2], '3': [3]}, observe_self=False,
         agent=dict(move_range=2, attack_range=2, attack_strength=0.5, attack_accuracy=0.6,
                    view_range=4, simultaneous_attacks=1)),
    dict(rows=9, cols=9, n_agents=30, n_teams=2, stacked_attacks=True,
         agent=dict(move_range=1, attack_range=1, attack_strength=0.4, attack_accuracy=0.9,
                    view_range=2, simultaneous_attacks=3)),
])
def test_dense_configs(oracle_mod, kw):
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=512, T=150, horizon=40, seed_run=5, key=3, as_list=True)


@pytest.mark.parametrize('kw', [
    dict(overlap={}),
    dict(no_overlap_at_reset=True),
    dict(rows=8, cols=8, n_agents=60, n_teams=3, overlap={}),   # 4 cells left for the last
    dict(rows=6, cols=11, n_agents=64, n_teams=4, no_overlap_at_reset=True),
])
def test_shared_list_placement(oracle_mod, kw):
    """Every placed cell leaves every list (no overlapping, or
    no_overlap_at_reset): the placement decodes the draws as a Lehmer code
    (gw_engine.hip do_reset, `shared`) -- against the oracle's sequential
    PositionState.reset, resets every few steps."""
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=1024, T=60, horizon=7, seed_run=14, key=31, check_every=1)


@pytest.mark.parametrize('kw', [
    # 128 BattleAgents on 32x32 (the headline grid with twice the fighters)
    dict(rows=32, cols=32, n_agents=128, n_teams=2),
    # 200 fighters, 4 teams, accuracy < 1, stacked double attacks, range 2
    dict(rows=24, cols=24, n_agents=200, n_teams=4, stacked_attacks=True,
         agent=dict(move_range=1, attack_range=2, attack_strength=0.5, attack_accuracy=0.7,
                    view_range=3, simultaneous_attacks=2)),
])
def test_team_battle_beyond_one_wave(oracle_mod, kw):
    """TeamBattle with more than 64 fighters: the workgroup-per-env kernel vs
    the oracle at 1024 envs."""
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=1024, T=120, horizon=60, seed_run=12, key=29, check_every=2, as_list=True)


@pytest.mark.parametrize('idx', [0, 3])
def test_dense_configs_workgroup_kernel(oracle_mod, idx):
    """Dense TeamBattle configs forced through the workgroup kernel."""
    kw = [dict(rows=8, cols=8, n_agents=16, n_teams=2),
          None, None,
          dict(rows=9, cols=9, n_agents=30, n_teams=2, stacked_attacks=True,
               agent=dict(move_range=1, attack_range=1, attack_strength=0.4, attack_accuracy=0.9,
                          view_range=2, simultaneous_attacks=3))][idx]
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=512, T=150, horizon=40, seed_run=5, key=3, force_workgroup=True, as_list=True)


@pytest.mark.parametrize('waves', [2, 4])
def test_headline_config_multi_wave(oracle_mod, waves):
    """The headline TeamBattle config on the workgroup kernel with 2 and 4
    waves per env (gw_config.force_workgroup = waves: the small-batch
    variant; threads past the 64 lanes share the table, store and crowded
    draws) vs the oracle."""
    cc = team_battle()
    _run(oracle_mod, cc, E=512, T=120, horizon=50, seed_run=3, key=17, check_every=2, force_workgroup=waves)


@pytest.mark.parametrize('kernel', ['lane', 'wave'])
def test_maze_navigation_1024_envs(oracle_mod, kernel):
    """BASELINE config 2: MazeNavigation 16x16 (generate_maze walls, blocking),
    1 navigator, 1024 envs, random moves, horizon auto-reset; on the
    one-lane-per-env kernel (the default for this config) and the one-wave
    kernel."""
    from abmarl_amd import _abi
    cc = build_maze(load_golden('maze_16')['case']).compiled()
    _run(oracle_mod, cc, E=1024, T=300, horizon=120, seed_run=2, key=5,
         env_per_lane=0 if kernel == 'lane' else -1,
         kernel=_abi.GW_KERNEL_LANE if kernel == 'lane' else _abi.GW_KERNEL_WAVE)


def test_maze_navigation_ammo_navigator(oracle_mod):
    """An AmmoAgent navigator (with an AmmoState): the lane-per-env kernel
    keeps no ammo, so the config runs on the one-wave kernel, whose reset is
    AmmoState.reset -- every env's navigator holds its initial_ammo."""
    import torch
    from abmarl_amd import _abi
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    from abmarl_amd.examples import MazeNavigationSim, MazeNavigationAgent
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent, AmmoAgent

    class AmmoNavigator(MazeNavigationAgent, AmmoAgent):
        pass

    c = load_golden('maze_16')['case']
    reg = {'N': lambda n: AmmoNavigator(id='navigator', encoding=1, view_range=c['agent']['view_range'],
                                        initial_ammo=7),
           'T': lambda n: GridWorldAgent(id='target', encoding=3),
           'W': lambda n: GridWorldAgent(id=f'wall{n}', encoding=2, blocking=True)}
    sim = MazeNavigationSim.build_sim_from_array(
        np.array(c['maze'], dtype=object), reg, overlapping={1: {3}, 3: {1}},
        states={'PositionState', 'AmmoState'}, observers={'PositionCenteredEncodingObserver'})
    cc = sim.compiled()
    eng = GridWorldEngine(cc, 64, seeds=env_seeds(64))
    assert eng.kernel == _abi.GW_KERNEL_WAVE
    eng.reset()
    lane = list(eng.lane_entities).index(list(sim.agents).index('navigator'))
    assert (eng.get_ammo().cpu().numpy()[:, lane] == 7).all()
    torch.cuda.synchronize()
    _run(oracle_mod, cc, E=512, T=150, horizon=60, seed_run=4, key=6, kernel=_abi.GW_KERNEL_WAVE)


@pytest.mark.parametrize('kw', [
    # TargetDestroyedDone (+ ActiveDone): hunt the next fighter of the other team
    dict(rows=12, cols=12, n_agents=30, n_teams=2, dones=['ActiveDone', 'TargetDestroyedDone'],
         target_mapping={f'agent{i}': f'agent{(i + 1) % 30}' for i in range(30)},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.8,
                    view_range=3)),
    # TargetAgentDone alone, cross-team overlap: chasers end on their target's cell
    dict(rows=8, cols=8, n_agents=16, n_teams=2, dones=['TargetAgentDone'],
         overlap={'1': [1, 2], '2': [2]},
         target_mapping={f'agent{i}': f'agent{(i + 5) % 16}' for i in range(16)},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.3, attack_accuracy=1,
                    view_range=2)),
])
def test_target_done_configs(oracle_mod, kw):
    """TeamBattle with the target done components (done.py:59-137) at 1024 envs."""
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=1024, T=150, horizon=60, seed_run=8, key=13)


@pytest.mark.parametrize('case', ['traffic_ex', 'traffic_9'])
def test_traffic_corridor_configs(oracle_mod, case):
    """TrafficCorridor (traffic_corridor.py, TargetAgentDone) at 1024 envs."""
    from tests.cases import build_traffic
    cc = build_traffic(load_golden(case)['case']).compiled()
    _run(oracle_mod, cc, E=1024, T=200, horizon=60, seed_run=9, key=17)


@pytest.mark.parametrize('kw', [
    # view ranges 1..4 mixed, blocking fighters and static walls (slot-geometry LUTs)
    dict(rows=16, cols=16, n_agents=40, n_teams=2, wall_encoding=3, blocking=list(range(0, 40, 4)),
         walls=[[r, 7] for r in range(2, 12)] + [[4, c] for c in range(9, 15)], views=[1, 4, 2, 3],
         agent=dict(move_range=1, attack_range=2, attack_strength=0.5, attack_accuracy=0.8,
                    view_range=3)),
    # observe_self=False, cross-team overlap (crowded cells with the observer's own cell)
    dict(rows=10, cols=10, n_agents=36, n_teams=3, views=[2, 1, 3], observe_self=False,
         overlap={'1': [1, 2], '2': [2], '3': [3, 1]}),
])
def test_mixed_view_configs(oracle_mod, kw):
    """Observers with different view ranges (observer.py:162-174) at 1024 envs."""
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=1024, T=120, horizon=50, seed_run=12, key=21)


@pytest.mark.parametrize('kw', [
    # static blocking walls + blocking fighters, attack range 2 (attack mask)
    dict(rows=16, cols=16, n_agents=40, n_teams=2, wall_encoding=3, blocking=list(range(0, 40, 3)),
         walls=[[r, 7] for r in range(2, 12)] + [[4, c] for c in range(9, 15)] + [[12, 2], [13, 13]],
         agent=dict(move_range=1, attack_range=2, attack_strength=0.5, attack_accuracy=0.8,
                    view_range=3)),
    # view 5 (two mask words per window), three teams, cross-team overlap
    dict(rows=20, cols=20, n_agents=48, n_teams=3, wall_encoding=4, blocking=[1, 2, 7, 20],
         overlap={'1': [1, 2], '2': [2], '3': [3]},
         walls=[[r, c] for r in range(3, 17, 4) for c in range(2, 18, 3)],
         agent=dict(move_range=2, attack_range=3, attack_strength=0.6, attack_accuracy=0.7,
                    view_range=5, simultaneous_attacks=2)),
])
def test_blocking_configs(oracle_mod, kw):
    cc = team_battle(**kw)
    _run(oracle_mod, cc, E=512, T=150, horizon=50, seed_run=7, key=9, as_list=True)


def test_generic_window_resets_cross_the_twist(oracle_mod):
    """The generic-window kernels (view 8: window side 17 > 15, so
    reset_kernel<0> / step_kernel<0, 0>, whose Rng and Smem live in scratch
    behind the out-of-line observe_big) on 64 random-health fighters: every
    reset draws 128 health words and the placement's, so a third of the
    resets cross the MT19937 twist in the health reset and in the placement
    -- the sites that read the key through a generic pointer (FLAT) until
    round 5 (DESIGN §4 "MT19937 key addressing")."""
    cc = team_battle(rows=20, cols=20, n_agents=64, n_teams=2,
                     agent=dict(move_range=1, attack_range=1, attack_strength=1, attack_accuracy=1,
                                view_range=8))
    assert cc.obs_side == 17            # > 2 * GW_FIXED_RANGE + 1: the generic window path
    _run(oracle_mod, cc, E=256, T=120, horizon=25, seed_run=5, key=31, check_every=3)


def test_next_step_autoreset_4096_envs(oracle_mod):
    """gw_step_autoreset_next on the headline config: envs whose episode ended
    in the previous call are reset (reward 0, done only for non-Agents, actions
    ignored), the others step; checked against the oracle doing exactly that."""
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc = team_battle()
    E, T, horizon = 4096, 150, 60
    seeds = env_seeds(E, run=3)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    NE, ln = cc.n_agents, eng.lane_entities
    o_obs = orc.new_obs()
    orc.reset(o_obs)
    assert (eng.reset().cpu().numpy() == o_obs[:, ln]).all()
    eng.all_done.zero_()
    rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8)
    ad = np.zeros(E, np.uint8)
    h_act = np.zeros((E, NE, 3), np.int32)
    resets = 0
    for t in range(T):
        act = eng.random_actions(17, t)
        h_act[:, ln] = act.cpu().numpy()
        rs = (ad != 0) | (orc.state()['steps'] >= horizon)
        resets += int(rs.sum())
        if rs.any():
            orc.reset(o_obs, mask=rs.astype(np.uint8))
        orc.step(h_act, o_obs, rew, done, ad, mask=(~rs).astype(np.uint8))
        live = (orc.state()['flags'] >> 1) & 1
        rew[rs] = 0.0
        done[rs] = 1 - live[rs]
        ad[rs] = 0
        obs, r, d, a = eng.step_autoreset_next(act, horizon=horizon)
        assert (a.cpu().numpy() == ad).all(), f"step {t}: __all__"
        assert (r.cpu().numpy().view(np.uint64) == rew[:, ln].view(np.uint64)).all(), f"step {t}: reward"
        assert (d.cpu().numpy() == done[:, ln]).all(), f"step {t}: done"
        g = obs.cpu().numpy()
        bad = g != o_obs[:, ln]
        assert not bad.any(), f"step {t}: obs mismatch at {np.argwhere(bad)[:3].tolist()}"
    torch.cuda.synchronize()
    assert resets > E // 2, resets
    st = eng.get_state()
    ost = orc.state()
    assert (st['pos'].cpu().numpy() == ost['pos'][:, ln]).all()
    mt = st['mt'].cpu().numpy().view(np.uint32)
    assert (mt[:, :625] == ost['mt'][:, :625]).all(), "RNG state"


RTT_WAVE_CASES = [
    # ReachTheTarget at the lane limit: 20 barriers + 40 runners + the target
    dict(rows=32, cols=32, n_barriers=20, n_runners=40,
         runner=dict(move_range=2, view_range=3),
         target=dict(view_range=3, attack_range=2, attack_strength=0.5, attack_accuracy=0.9,
                     simultaneous_attacks=2)),
    # crowded: runners start on the target's cell (double removes happen)
    dict(rows=6, cols=6, n_barriers=4, n_runners=20,
         runner=dict(move_range=1, view_range=2, initial_health=1),
         target=dict(view_range=2, attack_range=1, attack_strength=1, attack_accuracy=1)),
]


def _run_rtt(oracle_mod, kw, E, T, horizon, run=11, key=23, min_errs=0, force_workgroup=False):
    """ReachTheTarget (SelectiveAttackActor, TargetDone, OnlyAgentLeftDone)
    engine vs oracle; an env whose step raised (double remove) is reset by both."""
    from tests.cases import build_rtt
    cc = build_rtt(dict(kind='rtt', **kw)).compiled()
    return _run_raising(oracle_mod, cc, E, T, horizon, run, key, min_errs, force_workgroup, flag=4)


def _run_raising(oracle_mod, cc, E, T, horizon, run, key, min_errs=0, force_workgroup=False, flag=4):
    """Engine vs oracle for a program whose step can raise (err `flag`: 4 the
    double remove's KeyError, 32 the attack's ValueError): the raising envs'
    flags and RNG must agree, then both reset them."""
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc.cfg.force_workgroup = int(force_workgroup)
    seeds = env_seeds(E, run=run)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    NE, ln = cc.n_agents, eng.lane_entities
    o_obs = orc.new_obs()
    orc.reset(o_obs)
    assert (eng.reset().cpu().numpy() == o_obs[:, ln]).all()
    rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8); ad = np.zeros(E, np.uint8)
    h_act = np.zeros((E, NE, cc.act_dim), np.int32)
    errs = 0
    for t in range(T):
        act = eng.random_actions(key, t)
        h_act[:, ln] = act.cpu().numpy()
        eng.err.zero_()
        orc.step(h_act, o_obs, rew, done, ad)
        obs, r, d, a = eng.step(act)
        e_err = (eng.err.cpu().numpy() & flag) != 0
        o_err = (orc.errors() & flag) != 0
        assert (e_err == o_err).all(), f"step {t}: error flags"
        assert not ((eng.err.cpu().numpy() | orc.errors()) & ~flag).any(), f"step {t}: other flags"
        ok = ~o_err
        errs += int(o_err.sum())
        assert (a.cpu().numpy()[ok] == ad[ok]).all(), f"step {t}: __all__"
        assert (r.cpu().numpy().view(np.uint64)[ok] == rew[:, ln].view(np.uint64)[ok]).all(), f"step {t}: reward"
        assert (d.cpu().numpy()[ok] == done[:, ln][ok]).all(), f"step {t}: done"
        g = obs.cpu().numpy()
        bad = (g != o_obs[:, ln]) & ok[:, None, None, None]
        assert not bad.any(), f"step {t}: obs mismatch at {np.argwhere(bad)[:3].tolist()}"
        mt = eng.get_state()['mt'].cpu().numpy().view(np.uint32)
        assert (mt[:, :625] == orc.state()['mt'][:, :625]).all(), f"step {t}: RNG"
        rs = (ad != 0) | o_err | (orc.state()['steps'] >= horizon)
        if rs.any():
            m8 = rs.astype(np.uint8)
            orc.reset(o_obs, mask=m8)
            g = eng.reset(mask=torch.as_tensor(m8, device=eng.device)).cpu().numpy()
            assert (g[rs] == o_obs[:, ln][rs]).all(), f"step {t}: reset obs"
    st, ost = eng.get_state(), orc.state()
    assert (st['pos'].cpu().numpy() == ost['pos'][:, ln]).all()
    assert (st['health'].cpu().numpy() == ost['health'][:, ln]).all()
    assert (st['flags'].cpu().numpy() & 7 == ost['flags'][:, ln]).all()
    assert errs >= min_errs, errs
    return eng


@pytest.mark.parametrize('kernel', ['wave', 'wg'])
@pytest.mark.parametrize('case', [0, 1])
def test_reach_the_target_configs(oracle_mod, case, kernel):
    """Both ReachTheTarget kernels on the same configs (the workgroup kernel
    forced with gw_config.force_workgroup)."""
    eng = _run_rtt(oracle_mod, RTT_WAVE_CASES[case], E=512, T=120, horizon=40,
                   min_errs=1 if case == 1 else 0, force_workgroup=kernel == 'wg')
    assert eng.wg == (kernel == 'wg')


def test_reach_the_target_config4(oracle_mod):
    """BASELINE config 4 at one GPU's share of 8192 envs (1024): 64x64, 128
    barriers + 127 runners + the target = 256 lanes, the workgroup kernel."""
    from tests.cases import RTT_CONFIG4
    kw = {k: v for k, v in RTT_CONFIG4.items() if k != 'kind'}
    eng = _run_rtt(oracle_mod, kw, E=1024, T=60, horizon=25, run=4)
    assert eng.wg and eng.A == 256
    # the 1024-env launch in ONE dispatch round on the 256 CUs: 4 resident
    # workgroups (of 4 waves) per CU -- <= 128 VGPRs and <= 40 KiB of LDS
    import torch
    nblk, threads, lds = eng.step_occupancy()
    cus = torch.cuda.get_device_properties(eng.device).multi_processor_count
    assert threads == 256 and lds <= 160 * 1024 // 4, (threads, lds)
    assert nblk >= 4 and nblk * cus >= 1024, (nblk, cus)


def test_reach_the_target_config4_all_8192_envs(oracle_mod):
    """The bench's 'all 8192 envs on one GPU' launch shape of config 4
    (bench.py other_configs.reach_the_target_64_all_8192) vs the oracle."""
    from tests.cases import RTT_CONFIG4
    kw = {k: v for k, v in RTT_CONFIG4.items() if k != 'kind'}
    eng = _run_rtt(oracle_mod, kw, E=8192, T=24, horizon=12, run=13)
    assert eng.wg and eng.A == 256 and eng.E == 8192


@pytest.mark.parametrize('kw', [
    # random health, partial accuracy, 2 attacks per cell, crowded: 211 lanes
    dict(rows=24, cols=24, n_barriers=60, n_runners=150,
         runner=dict(move_range=1, view_range=2),
         target=dict(view_range=2, attack_range=2, attack_strength=0.5, attack_accuracy=0.7,
                     simultaneous_attacks=2)),
    # runners may not enter barrier cells: Grid.query can refuse a move, so
    # the move pass runs serially (one workgroup OR per mover)
    dict(rows=20, cols=20, n_barriers=50, n_runners=100, overlapping={'2': [3], '3': [2, 3]},
         runner=dict(move_range=2, view_range=3, initial_health=1),
         target=dict(view_range=3, attack_range=1, attack_strength=1, attack_accuracy=1)),
    # double removes at 150 lanes (runners start on the target's cell)
    dict(rows=8, cols=8, n_barriers=10, n_runners=139,
         runner=dict(move_range=1, view_range=2, initial_health=1),
         target=dict(view_range=2, attack_range=1, attack_strength=1, attack_accuracy=1)),
])
def test_reach_the_target_wide(oracle_mod, kw):
    eng = _run_rtt(oracle_mod, kw, E=256, T=80, horizon=30, run=5,
                   min_errs=1 if kw['rows'] == 8 else 0)
    assert eng.wg


def test_reach_the_target_config4_autoreset(oracle_mod):
    """Config 4 with NEXT_STEP and SAME_STEP auto-reset against the oracle.
    A step that raised (double remove) writes no reward/done; the auto-reset
    modes reset that env like an ended episode (all_done = 1; SAME_STEP
    returns the new episode's first observation in the same launch)."""
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    from tests.cases import build_rtt, RTT_CONFIG4
    cc = build_rtt(dict(RTT_CONFIG4)).compiled()
    E, T, horizon = 256, 50, 20
    for mode in ('next', 'same'):
        seeds = env_seeds(E, run=9)
        eng = GridWorldEngine(cc, E, seeds=seeds)
        orc = oracle_mod.Oracle(cc, E)
        orc.seed(seeds)
        NE, ln = cc.n_agents, eng.lane_entities
        o_obs = orc.new_obs()
        orc.reset(o_obs)
        assert (eng.reset().cpu().numpy() == o_obs[:, ln]).all()
        eng.all_done.zero_()
        rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8); ad = np.zeros(E, np.uint8)
        h_act = np.zeros((E, NE, cc.act_dim), np.int32)
        errs = 0
        for t in range(T):
            act = eng.random_actions(31, t)
            h_act[:, ln] = act.cpu().numpy()
            eng.err.zero_()
            if mode == 'next':
                rs = (ad != 0) | (orc.state()['steps'] >= horizon)
                if rs.any():
                    orc.reset(o_obs, mask=rs.astype(np.uint8))
                orc.step(h_act, o_obs, rew, done, ad, mask=(~rs).astype(np.uint8))
                o_err = ((orc.errors() & 4) != 0) & ~rs
                live = (orc.state()['flags'] >> 1) & 1
                rew[rs] = 0.0
                done[rs] = 1 - live[rs]
                ad[rs] = 0
                ad[o_err] = 1
                obs, r, d, a = eng.step_autoreset_next(act, horizon=horizon)
            else:
                orc.step(h_act, o_obs, rew, done, ad)
                o_err = (orc.errors() & 4) != 0
                ad[o_err] = 1
                rsm = (ad != 0) | (orc.state()['steps'] >= horizon)
                if rsm.any():
                    orc.reset(o_obs, mask=rsm.astype(np.uint8))
                obs, r, d, a = eng.step_autoreset(act, horizon=horizon)
            assert (((eng.err.cpu().numpy() & 4) != 0) == o_err).all(), f"{mode} step {t}: KeyError flags"
            ok = ~o_err
            errs += int(o_err.sum())
            assert (a.cpu().numpy() == ad).all(), f"{mode} step {t}: __all__"
            assert (r.cpu().numpy().view(np.uint64)[ok] == rew[:, ln].view(np.uint64)[ok]).all(), \
                f"{mode} step {t}: reward"
            assert (d.cpu().numpy()[ok] == done[:, ln][ok]).all(), f"{mode} step {t}: done"
            g = obs.cpu().numpy()
            cmp = ok if mode == 'next' else np.ones(E, bool)
            assert (g[cmp] == o_obs[:, ln][cmp]).all(), f"{mode} step {t}: obs"
        mt = eng.get_state()['mt'].cpu().numpy().view(np.uint32)
        assert (mt[:, :625] == orc.state()['mt'][:, :625]).all(), f"{mode}: RNG"
        assert errs > 0, "config 4 places runners on the target's cell: some steps raise"


@pytest.mark.parametrize('force_workgroup', [False, True])
@pytest.mark.parametrize('kw', [
    # simultaneous_attacks 3, accuracy < 1: np.random.choice's array of 2 or 3
    # picks whenever there are at least as many candidates as attacks
    dict(rows=8, cols=8, n_agents=40, n_teams=2, overlap={'1': [1, 2], '2': [2, 1]},
         agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.8,
                    view_range=2, simultaneous_attacks=3)),
    # stacked: an array for any candidate count
    dict(rows=10, cols=10, n_agents=30, n_teams=3, stacked_attacks=True,
         agent=dict(move_range=1, attack_range=2, attack_strength=0.4, attack_accuracy=1,
                    view_range=3, simultaneous_attacks=2)),
])
def test_team_battle_value_error(oracle_mod, kw, force_workgroup):
    """The reference's TeamBattleSim.step raises ValueError on `not
    attacked_agents` when BinaryAttackActor returns np.random.choice's array
    of 2 or more agents (team_battle_example.py:41, actor.py:412-414): both
    kernels flag GW_ERR_VALUE_ERROR at that attacker, with the attack's damage
    and draws applied and the step stopped, as the oracle does."""
    cc = team_battle(**kw)
    _run_raising(oracle_mod, cc, E=1024, T=60, horizon=30, run=21, key=41, min_errs=50,
                 force_workgroup=force_workgroup, flag=32)


def test_team_battle_value_error_opt_out(oracle_mod):
    """gw_config.attack_array_as_list = 1 (a simulation with
    attack_array_as_list = True): the list reading, no raise."""
    cc = team_battle(rows=8, cols=8, n_agents=40, n_teams=2, overlap={'1': [1, 2], '2': [2, 1]},
                     agent=dict(move_range=1, attack_range=1, attack_strength=0.5, attack_accuracy=0.8,
                                view_range=2, simultaneous_attacks=3))
    _run(oracle_mod, cc, E=1024, T=60, horizon=30, seed_run=21, key=41, as_list=True)


def test_timed_launch_shape_vs_oracle(oracle_mod):
    """The driver's timed launch, pinned to the oracle directly (not through
    single steps): bench.py's headline workload -- 4096 envs of the 32x32 /
    64-agent TeamBattle, seeds env_seeds(run=0), the first episode of env e
    starting at step e * 200 // 4096, horizon 200 -- a 220-step pre-roll as
    gw_rollout fragments, then two 20-step fragments (the timed launch's
    size), all with skip_done_obs and NEXT_STEP auto-reset, on the bench's
    Philox actions.  Every step of every fragment is compared with the oracle
    running the same protocol: each written obs row (the rows of agents that
    get an observation), reward bits, dones, __all__; then the state and the
    RNG."""
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    from tests.cases import team_battle
    cc = team_battle()
    E, H, key = 4096, 200, 0x5eed0000
    seeds = env_seeds(E, run=0)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    NE, ln = cc.n_agents, eng.lane_entities
    o_obs = orc.new_obs()
    orc.reset(o_obs)
    assert (eng.reset().cpu().numpy() == o_obs[:, ln]).all(), "reset obs"
    eng.all_done.zero_()
    stagger = (np.arange(E) * H // E).astype(np.int32)
    eng.set_state(steps=torch.as_tensor(stagger, device=eng.device))
    orc.set_steps(stagger)
    rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8); ad = np.zeros(E, np.uint8)
    h_act = np.zeros((E, NE, 3), np.int32)
    frags = [50, 50, 50, 50, 20, 20, 20]          # 220 pre-roll steps, then the timed launch twice
    t = resets = rows = 0
    for f in frags:
        acts = torch.empty((f,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
        for s in range(f):
            eng.random_actions(key, t + s, out=acts[s])
        out = eng.rollout(acts, horizon=H, autoreset='next_step', skip_done_obs=True)
        g_obs, g_rew = out['obs'].cpu().numpy(), out['reward'].cpu().numpy()
        g_done, g_ad = out['done'].cpu().numpy(), out['all_done'].cpu().numpy()
        h_all = acts.cpu().numpy()
        for s in range(f):
            h_act[:, ln] = h_all[s]
            rs = (ad != 0) | (orc.state()['steps'] >= H)          # NEXT_STEP: reset instead of step
            resets += int(rs.sum())
            if rs.any():
                orc.reset(o_obs, mask=rs.astype(np.uint8))
            orc.step(h_act, o_obs, rew, done, ad, mask=(~rs).astype(np.uint8))
            live = (orc.state()['flags'] >> 1) & 1
            rew[rs] = 0.0
            done[rs] = 1 - live[rs]
            ad[rs] = 0
            where = f"step {t + s} (fragment of {f})"
            assert (g_ad[s] == ad).all(), f"{where}: __all__"
            assert (g_rew[s].view(np.uint64) == rew[:, ln].view(np.uint64)).all(), f"{where}: reward"
            assert (g_done[s] == done[:, ln]).all(), f"{where}: done"
            want = o_obs[:, ln]
            m = (want != -2).reshape(E, len(ln), -1).any(-1)        # the rows written this step
            rows += int(m.sum())
            bad = g_obs[s][m] != want[m]
            assert not bad.any(), f"{where}: obs mismatch in {int(bad.any(-1).any(-1).sum())} rows"
        t += f
    torch.cuda.synchronize()
    assert resets > E // 2, resets            # horizon ends and __all__ inside the fragments
    st, ost = eng.get_state(), orc.state()
    assert (st['pos'].cpu().numpy() == ost['pos'][:, ln]).all()
    assert (st['health'].cpu().numpy() == ost['health'][:, ln]).all()
    assert (st['flags'].cpu().numpy() & 7 == ost['flags'][:, ln]).all()
    assert (st['steps'].cpu().numpy() == ost['steps']).all()
    mt = st['mt'].cpu().numpy().view(np.uint32)
    assert (mt[:, :625] == ost['mt'][:, :625]).all(), "RNG state"
    assert not eng.err.any().item()
    assert rows > 220 * E * 20, rows
