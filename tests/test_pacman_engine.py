"""The HIP Pacman program (abmarl_amd/csrc/gw_pacman.inc) on the GPU:
  * AllStepManager protocol, batched and through the dict API, against the
    reference's own trajectories (tests/golden/pacman_*.npz);
  * TurnBasedManager protocol (BASELINE config 5, build-defined: the
    reference cannot run it) against the C oracle at scale, and the dict API
    under our TurnBasedManager against the oracle;
  * same-step / next-step auto-reset at scale against the oracle."""
import json
import os
import zlib

import numpy as np
import pytest

from abmarl_amd import _abi

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    z = np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d['case'] = json.loads(str(d['case']))
    return d


def _sim(c=None):
    from abmarl_amd.examples.pacman import build_pacman
    if c is None:
        return build_pacman()
    return build_pacman(baddies=c['baddies'], reward_scheme=c['reward_scheme'])


def _food_bits(words, n):
    w = words.view(np.uint32)
    return np.array([[(w[e, k >> 5] >> (k & 31)) & 1 for k in range(n)] for e in range(w.shape[0])],
                    np.uint8)


@pytest.mark.parametrize('name', ['pacman_4', 'pacman_10'])
def test_batched_allstep_matches_reference(name):
    import torch
    from abmarl_amd.engine import GridWorldEngine
    g = load(name)
    c = g['case']
    cc = _sim(c).compiled()
    E, T = c['n_envs'], c['n_steps']
    eng = GridWorldEngine(cc, E, seeds=np.array(c['seeds'], np.uint32))
    assert list(eng.lane_entities) == c['agent_index']
    assert eng.obs_shape == (21, 21) and eng.n_passive == len(c['food_index'])
    assert (eng.reset().cpu().numpy() == g['obs0']).all()
    act = torch.zeros_like(eng.actions)
    for t in range(T):
        act[:, :, 0] = torch.as_tensor(g['actions'][t].astype(np.int32), device=eng.device)
        obs, r, d, a = eng.step(act)
        obs, r, d, a = obs.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(), a.cpu().numpy()
        ret = g['returned'][t].astype(bool)
        assert (obs[ret] == g['obs'][t][ret]).all(), f"step {t}: obs"
        assert (r[ret].view(np.uint64) == g['reward'][t][ret].view(np.uint64)).all(), f"step {t}: reward"
        assert (d[ret] == g['done'][t][ret]).all(), f"step {t}: done"
        assert (a == g['all_done'][t]).all(), f"step {t}: __all__"
        st, aux = eng.get_state(), eng.get_aux_state()
        assert (st['pos'].cpu().numpy() == g['pos'][t]).all(), f"step {t}: positions"
        assert ((st['flags'].cpu().numpy() >> 3) & 7 == g['orient'][t]).all(), f"step {t}: orientation"
        assert (_food_bits(aux['passive'].cpu().numpy(), eng.n_passive) == g['food'][t]).all(), \
            f"step {t}: food"
        mt = st['mt'].cpu().numpy().view(np.uint32)
        assert (mt[:, _abi.GW_MT_N] == g['mt_pos'][t]).all(), f"step {t}: RNG position"
        assert [zlib.crc32(np.ascontiguousarray(mt[e, :_abi.GW_MT_N]).tobytes())
                for e in range(E)] == g['mt_crc'][t].tolist(), f"step {t}: RNG key"
        rs = g['reset_mask'][t]
        if rs.any():
            o = eng.reset(mask=torch.as_tensor(rs, device=eng.device)).cpu().numpy()
            assert (o[rs.astype(bool)] == g['reset_obs'][t][rs.astype(bool)]).all(), f"step {t}: reset"


@pytest.mark.parametrize('name', ['pacman_4', 'pacman_shuffle_act'])
def test_dict_allstep_matches_reference(name):
    """build_pacman + AllStepManager, np.random.seed per env, as the reference;
    pacman_shuffle_act: AllStepManager(randomize_action_input=True), the
    baddies moving in the shuffled dict's order (Python's random per env)."""
    import random
    from abmarl_amd.managers import AllStepManager
    g = load(name)
    c = g['case']
    for e in range(2):
        sim = _sim(c)
        ids = list(sim.agents)
        agents = [ids[i] for i in c['agent_index']]
        m = AllStepManager(sim, randomize_action_input=bool(c.get('randomize_action_input', False)))
        np.random.seed(c['seeds'][e])
        if 'py_seeds' in c:
            random.seed(c['py_seeds'][e])
        o = m.reset()
        for j, aid in enumerate(agents):
            assert (o[aid]['absolute_encoding'] == g['obs0'][e, j]).all()
        steps = 0
        for t in range(c['n_steps']):
            adict = {aid: {'move': int(g['actions'][t, e, j])} for j, aid in enumerate(agents)
                     if aid not in m.done_agents}
            o, r, d, _ = m.step(adict)
            steps += 1
            for j, aid in enumerate(agents):
                if g['returned'][t, e, j]:
                    assert (o[aid]['absolute_encoding'] == g['obs'][t, e, j]).all(), (t, aid)
                    assert r[aid] == g['reward'][t, e, j], (t, aid)
                    assert d[aid] == bool(g['done'][t, e, j])
            assert d['__all__'] == bool(g['all_done'][t, e])
            st = np.random.get_state()
            assert st[2] == g['mt_pos'][t, e]
            assert zlib.crc32(np.ascontiguousarray(st[1], np.uint32).tobytes()) == g['mt_crc'][t, e]
            if g['reset_mask'][t, e]:
                o = m.reset()
                for j, aid in enumerate(agents):
                    assert (o[aid]['absolute_encoding'] == g['reset_obs'][t, e, j]).all()


def _turn_vs_oracle(oracle_mod, cc, E, T, horizon, key, seed_run):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    seeds = env_seeds(E, run=seed_run)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    ln = eng.lane_entities
    NE = cc.n_agents
    o_obs = orc.new_obs()
    o_ret, o_turn, _ = orc.turn_reset(o_obs)
    obs, ret, turn = eng.turn_reset()
    assert (turn.cpu().numpy() == np.searchsorted(ln, o_turn)).all()
    assert (ret.cpu().numpy() == o_ret[:, ln]).all()
    g = obs.cpu().numpy()
    r8 = o_ret[:, ln].astype(bool)
    assert (g[r8] == o_obs[:, ln][r8]).all()
    eng.all_done.zero_()
    rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8); ad = np.zeros(E, np.uint8)
    h_act = np.zeros((E, NE, cc.act_dim), np.int32)
    resets = steps = 0
    for t in range(T):
        act = eng.random_actions(key, t)
        h_act[:, ln] = act.cpu().numpy()
        rs = (ad != 0) | (orc.state()['steps'] >= horizon)
        m = (~rs).astype(np.uint8)
        o_ret = np.zeros((E, NE), np.uint8)
        o_turn = np.zeros(E, np.int32)
        if m.any():
            rr, tt = orc.turn_step(h_act, o_obs, rew, done, ad, mask=m)
            o_ret[m.astype(bool)] = rr[m.astype(bool)]
            o_turn[m.astype(bool)] = tt[m.astype(bool)]
            steps += int(m.sum())
        if rs.any():
            rr, tt, _ = orc.turn_reset(o_obs, mask=rs.astype(np.uint8))
            o_ret[rs] = rr[rs]
            o_turn[rs] = tt[rs]
            rew[rs] = 0.0
            done[rs] = 0
            ad[rs] = 0
            resets += int(rs.sum())
        obs, r, d, a, ret, turn = eng.turn_step(act, horizon=horizon)
        assert (a.cpu().numpy() == ad).all(), f"step {t}: __all__"
        assert (turn.cpu().numpy() == np.searchsorted(ln, o_turn)).all(), f"step {t}: turn"
        rt = ret.cpu().numpy()
        assert (rt == o_ret[:, ln]).all(), f"step {t}: returned"
        rb = rt.astype(bool)
        assert (r.cpu().numpy()[rb].view(np.uint64) == rew[:, ln][rb].view(np.uint64)).all(), \
            f"step {t}: reward"
        assert (d.cpu().numpy()[rb] == done[:, ln][rb]).all(), f"step {t}: done"
        g = obs.cpu().numpy()
        bad = (g != o_obs[:, ln]) & rb[:, :, None, None]
        assert not bad.any(), f"step {t}: obs mismatch at {np.argwhere(bad)[:3].tolist()}"
    torch.cuda.synchronize()
    st, ost = eng.get_state(), orc.state()
    assert (st['pos'].cpu().numpy() == ost['pos'][:, ln]).all()
    mt = st['mt'].cpu().numpy().view(np.uint32)
    assert (mt[:, :625] == ost['mt'][:, :625]).all(), "RNG state"
    return resets, steps


def test_turn_based_config5_vs_oracle(oracle_mod):
    """BASELINE config 5 (pacman.txt, 4 baddies, TurnBasedManager) batched,
    next-step auto-reset, random cross moves, 2048 envs."""
    cc = _sim().compiled()
    resets, steps = _turn_vs_oracle(oracle_mod, cc, E=2048, T=260, horizon=200, key=31, seed_run=4)
    assert resets > 0 and steps > 0


def test_turn_based_config5_16384_envs_vs_oracle(oracle_mod):
    """The bench's config 5 launch shape (16384 envs, TurnBasedManager,
    next-step auto-reset) for 60 turns, a short horizon so that resets land
    inside the run."""
    cc = _sim().compiled()
    resets, steps = _turn_vs_oracle(oracle_mod, cc, E=16384, T=60, horizon=25, key=37, seed_run=6)
    assert resets > 0 and steps > 0


def test_dict_turn_based_matches_oracle(oracle_mod):
    """TurnBasedManager over the engine-backed PacmanSim (dict API) against the
    oracle's turn protocol from the same np.random seed."""
    from abmarl_amd.managers import TurnBasedManager
    sim = _sim()
    cc = sim.compiled()
    ids = list(sim.agents)
    m = TurnBasedManager(sim)
    orc = oracle_mod.Oracle(cc, 1)
    orc.seed(np.array([123], np.uint32))
    o_obs = orc.new_obs()
    rew = np.zeros((1, cc.n_agents)); done = np.zeros((1, cc.n_agents), np.uint8)
    ad = np.zeros(1, np.uint8)
    np.random.seed(123)
    o = m.reset()
    o_ret, turn, _ = orc.turn_reset(o_obs)
    (aid, ob), = o.items()
    assert ids.index(aid) == turn[0]
    assert (ob['absolute_encoding'] == o_obs[0, turn[0]]).all()
    rs = np.random.RandomState(8)
    episodes = 0
    for t in range(300):
        mv = int(rs.randint(0, 5))
        act = np.zeros((1, cc.n_agents, cc.act_dim), np.int32)
        act[0, turn[0], 0] = mv
        o, r, d, _ = m.step({ids[turn[0]]: {'move': mv}})
        ret, turn = orc.turn_step(act, o_obs, rew, done, ad)
        assert sorted(o) == sorted(ids[i] for i in np.nonzero(ret[0])[0])
        for aid in o:
            i = ids.index(aid)
            assert (o[aid]['absolute_encoding'] == o_obs[0, i]).all(), (t, aid)
            assert r[aid] == rew[0, i] and d[aid] == bool(done[0, i])
        assert d['__all__'] == bool(ad[0])
        if ad[0]:
            episodes += 1
            (aid, ob), = m.reset().items()
            _, turn, _ = orc.turn_reset(o_obs)
            assert ids.index(aid) == turn[0]
            assert (ob['absolute_encoding'] == o_obs[0, turn[0]]).all()
            ad[0] = 0


@pytest.mark.parametrize('mode', ['same_step', 'next_step'])
def test_allstep_autoreset_vs_oracle(oracle_mod, mode):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc = _sim().compiled()
    E, T, horizon = 1024, 200, 90
    seeds = env_seeds(E, run=9)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    ln = eng.lane_entities
    NE = cc.n_agents
    o_obs = orc.new_obs()
    orc.reset(o_obs)
    assert (eng.reset().cpu().numpy() == o_obs[:, ln]).all()
    eng.all_done.zero_()
    rew = np.zeros((E, NE)); done = np.zeros((E, NE), np.uint8); ad = np.zeros(E, np.uint8)
    h_act = np.zeros((E, NE, cc.act_dim), np.int32)
    for t in range(T):
        act = eng.random_actions(5, t)
        h_act[:, ln] = act.cpu().numpy()
        if mode == 'same_step':
            orc.step(h_act, o_obs, rew, done, ad)
            orc.reset(o_obs, all_done=ad, horizon=horizon)
            obs, r, d, a = eng.step_autoreset(act, horizon=horizon)
        else:
            rs = (ad != 0) | (orc.state()['steps'] >= horizon)
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
    mt = eng.get_state()['mt'].cpu().numpy().view(np.uint32)
    assert (mt[:, :625] == orc.state()['mt'][:, :625]).all(), "RNG state"


def _pac_pair(E, run, stagger=0):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc = _sim().compiled()
    engs = [GridWorldEngine(cc, E, seeds=env_seeds(E, run=run)) for _ in range(2)]
    for eng in engs:
        eng.turn_reset()
        eng.all_done.zero_()
        if stagger:
            eng.set_state(steps=torch.as_tensor((np.arange(E) * stagger // E).astype(np.int32),
                                                device=eng.device))
    return engs


def _same_state(a, b):
    sa, sb = a.get_state(), b.get_state()
    for k in ('pos', 'health', 'flags', 'seq', 'steps'):
        assert (sa[k].cpu().numpy() == sb[k].cpu().numpy()).all(), k
    assert (sa['mt'].cpu().numpy()[:, :625] == sb['mt'].cpu().numpy()[:, :625]).all(), 'RNG'
    xa, xb = a.get_aux_state(), b.get_aux_state()
    for k in xa:
        assert (xa[k].cpu().numpy() == xb[k].cpu().numpy()).all(), k
    assert (a.acting.cpu().numpy() == b.acting.cpu().numpy()).all(), 'acting'
    assert (a.err.cpu().numpy() == b.err.cpu().numpy()).all(), 'err'


@pytest.mark.parametrize('E,frags,horizon', [(2048, (1, 17, 40, 100), 60), (16384, (50, 50), 200)])
def test_turn_rollout_matches_turn_steps(E, frags, horizon):
    """gw_turn_rollout (K turns in one launch) against K gw_turn_step calls on
    an engine with the same seeds, bit for bit: every turn's returned rows
    of obs, reward bits, done, returned, turn, __all__, then the engine
    state.  (gw_turn_step itself is pinned to the oracle above.)  16384
    envs with 50-turn fragments is the bench's config-5 launch shape."""
    import torch
    a, b = _pac_pair(E, run=11, stagger=horizon)
    t = 0
    for f in frags:
        acts = torch.empty((f,) + tuple(a.actions.shape), dtype=torch.int32, device=a.device)
        for s in range(f):
            a.random_actions(41, t + s, out=acts[s])
        out = a.turn_rollout(acts, horizon=horizon)
        for s in range(f):
            obs, r, d, ad, ret, turn = b.turn_step(acts[s].contiguous(), horizon=horizon)
            rt = ret.cpu().numpy()
            assert (out['returned'][s].cpu().numpy() == rt).all(), f"turn {t + s}: returned"
            assert (out['turn'][s].cpu().numpy() == turn.cpu().numpy()).all(), f"turn {t + s}: turn"
            assert (out['all_done'][s].cpu().numpy() == ad.cpu().numpy()).all(), f"turn {t + s}: __all__"
            assert (out['reward'][s].cpu().numpy().view(np.uint64) ==
                    r.cpu().numpy().view(np.uint64)).all(), f"turn {t + s}: reward"
            assert (out['done'][s].cpu().numpy() == d.cpu().numpy()).all(), f"turn {t + s}: done"
            rb = rt.astype(bool)
            assert (out['obs'][s].cpu().numpy()[rb] == obs.cpu().numpy()[rb]).all(), f"turn {t + s}: obs"
        t += f
    assert (a.all_done.cpu().numpy() == b.all_done.cpu().numpy()).all()
    assert (a.turn.cpu().numpy() == b.turn.cpu().numpy()).all()
    _same_state(a, b)


@pytest.mark.parametrize('mode', ['next_step', 'same_step'])
def test_allstep_rollout_matches_steps(mode):
    """gw_rollout on the Pacman program (one launch per fragment) against
    single AllStepManager steps with auto-reset, bit for bit."""
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    cc = _sim().compiled()
    E, horizon = 1024, 45
    a, b = [GridWorldEngine(cc, E, seeds=env_seeds(E, run=12)) for _ in range(2)]
    for eng in (a, b):
        eng.reset()
        eng.all_done.zero_()
    step_b = b.step_autoreset_next if mode == 'next_step' else b.step_autoreset
    t = 0
    for f in (1, 9, 64):
        acts = torch.empty((f,) + tuple(a.actions.shape), dtype=torch.int32, device=a.device)
        for s in range(f):
            a.random_actions(43, t + s, out=acts[s])
        out = a.rollout(acts, horizon=horizon, autoreset=mode)
        for s in range(f):
            obs, r, d, ad = step_b(acts[s].contiguous(), horizon=horizon)
            assert (out['all_done'][s].cpu().numpy() == ad.cpu().numpy()).all(), f"step {t + s}: __all__"
            assert (out['reward'][s].cpu().numpy().view(np.uint64) ==
                    r.cpu().numpy().view(np.uint64)).all(), f"step {t + s}: reward"
            assert (out['done'][s].cpu().numpy() == d.cpu().numpy()).all(), f"step {t + s}: done"
            assert (out['obs'][s].cpu().numpy() == obs.cpu().numpy()).all(), f"step {t + s}: obs"
        t += f
    _same_state(a, b)


def test_two_foods_on_one_cell_refused():
    """The Pacman program places every entity at its own initial cell and
    its cell -> food map holds one food per cell (gw_pacman.inc food_at):
    gw_create refuses a layout with two foods on a cell."""
    import numpy as np
    from abmarl_amd._native import EngineError
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    from abmarl_amd.examples.pacman import PacmanSim, PacmanAgent, FoodAgent, BaddieAgent
    agents = {
        'pacman': PacmanAgent(id='pacman', encoding=1, initial_position=np.array([0, 0])),
        'baddie_0': BaddieAgent(id='baddie_0', encoding=4, initial_position=np.array([4, 4])),
        'food_0': FoodAgent(id='food_0', encoding=3, initial_position=np.array([2, 2])),
        'food_1': FoodAgent(id='food_1', encoding=3, initial_position=np.array([2, 2])),
    }
    sim = PacmanSim.build_sim(5, 5, agents=agents,
                              states={'PositionState', 'OrientationState', 'HealthState'},
                              observers={'AbsoluteEncodingObserver'},
                              overlapping={1: {3, 4}, 3: {3}, 4: {3, 4}})
    with pytest.raises(EngineError, match='share initial cell|another food'):
        GridWorldEngine(sim.compiled(), 4, seeds=env_seeds(4))
