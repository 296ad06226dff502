"""HIP engine vs the C oracle at scale: the headline TeamBattle configuration
(32x32, 64 agents, 2 teams) with random-policy actions, in-launch auto-reset,
compared bit-exactly every step (obs, float64 reward bits, dones, __all__)
and on the final engine state (positions, health, flags, RNG)."""
import numpy as np
import pytest

from tests.cases import team_battle

pytestmark = pytest.mark.gpu


def _run(oracle_mod, cc, E, T, horizon, seed_run, key, check_every=1):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    seeds = env_seeds(E, run=seed_run)
    eng = GridWorldEngine(cc, E, seeds=seeds)
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(seeds)
    A = cc.n_agents
    o_obs = orc.new_obs()
    orc.reset(o_obs)
    g_obs = eng.reset().cpu().numpy()
    assert (g_obs == o_obs).all(), "reset obs"
    rew = np.zeros((E, A)); done = np.zeros((E, A), np.uint8); ad = np.zeros(E, np.uint8)
    for t in range(T):
        act = eng.random_actions(key, t)
        h_act = act.cpu().numpy()
        orc.step(h_act, o_obs, rew, done, ad)
        orc.reset(o_obs, all_done=ad, horizon=horizon)
        obs, r, d, a = eng.step_autoreset(act, horizon=horizon)
        assert (r.cpu().numpy().view(np.uint64) == rew.view(np.uint64)).all(), f"step {t}: reward"
        assert (d.cpu().numpy() == done).all(), f"step {t}: done"
        assert (a.cpu().numpy() == ad).all(), f"step {t}: __all__"
        if t % check_every == 0 or t == T - 1:
            g = obs.cpu().numpy()
            bad = g != o_obs
            assert not bad.any(), f"step {t}: obs mismatch at {np.argwhere(bad)[:3].tolist()}"
    torch.cuda.synchronize()
    st = eng.get_state()
    ost = orc.state()
    assert (st['pos'].cpu().numpy() == ost['pos']).all()
    assert (st['health'].cpu().numpy() == ost['health']).all()
    assert (st['flags'].cpu().numpy() == ost['flags']).all()
    mt = st['mt'].cpu().numpy().view(np.uint32)
    assert (mt[:, :625] == ost['mt'][:, :625]).all(), "RNG state"
    assert not eng.err.any().item()


def test_headline_config_4096_envs(oracle_mod):
    cc = team_battle()
    _run(oracle_mod, cc, E=4096, T=160, horizon=70, seed_run=0, key=11, check_every=4)


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
    _run(oracle_mod, cc, E=512, T=150, horizon=40, seed_run=5, key=3)
