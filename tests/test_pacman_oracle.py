"""The C oracle's Pacman program (oracle/gw_oracle.c pac_*) against the
reference's own PacmanSim + AllStepManager trajectories
(tests/golden/pacman_*.npz, made by tests/golden/make_pacman.py): absolute
observations, rewards (float64 bits), dones, positions, orientations, food,
RNG stream position and key digest, through resets."""
import json
import os
import zlib

import numpy as np
import pytest

from abmarl_amd import _abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    z = np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d['case'] = json.loads(str(d['case']))
    return d


def compiled(c):
    from abmarl_amd.examples.pacman import build_pacman
    sim = build_pacman(baddies=c['baddies'], reward_scheme=c['reward_scheme'])
    return sim.compiled()


@pytest.mark.parametrize('name', ['pacman_4', 'pacman_10'])
def test_oracle_matches_reference(oracle_mod, name):
    g = load(name)
    c = g['case']
    cc = compiled(c)
    E, T = c['n_envs'], c['n_steps']
    ag, food = c['agent_index'], c['food_index']
    assert cc.n_agents == c['n_entities']
    orc = oracle_mod.Oracle(cc, E)
    orc.seed(np.array(c['seeds'], np.uint32))
    obs = orc.new_obs()
    orc.reset(obs)
    assert (obs[:, ag] == g['obs0']).all()
    rew = np.zeros((E, cc.n_agents)); done = np.zeros((E, cc.n_agents), np.uint8)
    ad = np.zeros(E, np.uint8)
    act = np.zeros((E, cc.n_agents, cc.act_dim), np.int32)
    for t in range(T):
        act[:, ag, 0] = g['actions'][t]
        orc.step(act, obs, rew, done, ad)
        ret = g['returned'][t].astype(bool)
        for e in range(E):
            r = ret[e]
            assert (obs[e, ag][r] == g['obs'][t, e][r]).all(), f"step {t} env {e}: obs"
            assert (rew[e, ag][r].view(np.uint64) == g['reward'][t, e][r].view(np.uint64)).all(), \
                f"step {t} env {e}: reward {rew[e, ag][r]} vs {g['reward'][t, e][r]}"
            assert (done[e, ag][r] == g['done'][t, e][r]).all(), f"step {t} env {e}: done"
        assert (ad == g['all_done'][t]).all(), f"step {t}: __all__"
        st, aux = orc.state(), orc.aux()
        assert (st['pos'][:, ag] == g['pos'][t]).all(), f"step {t}: positions"
        assert (aux['orient'][:, ag] == g['orient'][t]).all(), f"step {t}: orientation"
        assert (((st['flags'][:, food] >> 2) & 1) == g['food'][t]).all(), f"step {t}: food"
        mt = st['mt']
        assert (mt[:, _abi.GW_MT_N] == g['mt_pos'][t]).all(), f"step {t}: RNG position"
        assert [zlib.crc32(np.ascontiguousarray(mt[e, :_abi.GW_MT_N]).tobytes())
                for e in range(E)] == g['mt_crc'][t].tolist(), f"step {t}: RNG key"
        rs = g['reset_mask'][t]
        if rs.any():
            orc.reset(obs, mask=rs)
            for e in np.nonzero(rs)[0]:
                assert (obs[e, ag] == g['reset_obs'][t, e]).all(), f"step {t} env {e}: reset obs"


def test_shuffled_pacman_is_order_invariant(oracle_mod):
    """pacman_shuffle_act (AllStepManager(randomize_action_input=True), the
    reference's own trajectory) replays in agents-dict order too: every
    baddie has encoding 4 and overlaps the others, so the order they move and
    stack in changes no observation, draw or reward bit.  The GPU replay
    (test_pacman_engine.py) still runs the shuffled order, which only has to
    leave the Python and numpy streams where the reference leaves them."""
    test_oracle_matches_reference(oracle_mod, 'pacman_shuffle_act')


class _OracleSim:
    """The oracle's simulation-only protocol (gwo_sim_*, gwo_observe,
    gwo_take_reward) behind the AgentBasedSimulation calls a manager makes,
    for one env — so the Python managers (pinned against the reference on
    MultiCorridor) can drive it."""

    def __init__(self, oracle_mod, cc, agents, seed):
        self.o = oracle_mod.Oracle(cc, 1)
        self.o.seed(np.array([seed], np.uint32))
        self.cc = cc
        self.agents = agents
        self.ids = list(agents)
        self.obs = self.o.new_obs()
        self._all = False

    def reset(self):
        self.o.sim_reset()
        self._all = False

    def step(self, action_dict):
        act = np.zeros((1, self.cc.n_agents, self.cc.act_dim), np.int32)
        act[0, :, 2] = -1
        for aid, a in action_dict.items():
            i = self.ids.index(aid)
            act[0, i, 0] = a['move']
            act[0, i, 2] = 0
        _, ad = self.o.sim_step(act)
        self._all = bool(ad[0])

    def get_obs(self, aid):
        i = self.ids.index(aid)
        self.o.observe(i, self.obs)
        return self.obs[0, i].copy()

    def get_reward(self, aid):
        return float(self.o.take_reward(self.ids.index(aid))[0])

    def get_done(self, aid):
        return self._all

    def get_all_done(self):
        return self._all

    def get_info(self, aid):
        return {}


def test_oracle_turn_protocol_matches_python_manager(oracle_mod):
    """gwo_turn_reset/gwo_turn_step (the batched TurnBasedManager the engine
    mirrors) against our Python TurnBasedManager driving the oracle's
    simulation-only protocol: same observations (hence the same draws),
    rewards, dones, turn order, through episode ends."""
    from abmarl_amd.examples.pacman import build_pacman
    from abmarl_amd.managers import TurnBasedManager
    from abmarl_amd.managers.simulation_manager import SimulationManager
    sim = build_pacman()
    cc = sim.compiled()
    ids = list(sim.agents)
    E, T = 3, 400
    seeds = [91, 92, 93]
    batched = oracle_mod.Oracle(cc, E)
    batched.seed(np.array(seeds, np.uint32))
    obs_b = batched.new_obs()
    rew = np.zeros((E, cc.n_agents)); done = np.zeros((E, cc.n_agents), np.uint8)
    ad = np.zeros(E, np.uint8)
    ret, turn, _ = batched.turn_reset(obs_b)
    rs = np.random.RandomState(4)
    mans = []
    for e in range(E):
        osim = _OracleSim(oracle_mod, cc, sim.agents, seeds[e])
        m = TurnBasedManager.__new__(TurnBasedManager)
        SimulationManager.__init__(m, sim)                 # the agents dict (kinds, order)
        from itertools import cycle
        from abmarl_amd.sim.agent_based_simulation import Agent
        m.agent_order = cycle([a for a, ag in sim.agents.items() if isinstance(ag, Agent)])
        m.sim = osim
        mans.append(m)
    first = [m.reset() for m in mans]
    for e in range(E):
        (aid, o), = first[e].items()
        assert ids.index(aid) == turn[e] and ret[e].sum() == 1
        assert (o == obs_b[e, ids.index(aid)]).all()
    episodes = 0
    for t in range(T):
        act = np.zeros((E, cc.n_agents, cc.act_dim), np.int32)
        moves = rs.randint(0, 5, size=E)
        for e in range(E):
            act[e, turn[e], 0] = moves[e]
        ret, turn_n = batched.turn_step(act, obs_b, rew, done, ad)
        for e in range(E):
            o, r, d, _ = mans[e].step({ids[turn[e]]: {'move': int(moves[e])}})
            got = [ids[i] for i in np.nonzero(ret[e])[0]]
            assert sorted(got) == sorted(o.keys()), (t, e)
            for aid in o:
                i = ids.index(aid)
                assert (o[aid] == obs_b[e, i]).all(), (t, e, aid)
                assert np.float64(r[aid]).view(np.uint64) == rew[e, i].view(np.uint64), (t, e, aid)
                assert bool(d[aid]) == bool(done[e, i])
            assert bool(d['__all__']) == bool(ad[e])
        turn = turn_n
        if ad.any():
            episodes += int(ad.sum())
            ret2, turn2, _ = batched.turn_reset(obs_b, mask=ad.copy())
            for e in np.nonzero(ad)[0]:
                (aid, o), = mans[e].reset().items()
                assert ids.index(aid) == turn2[e]
                assert (o == obs_b[e, turn2[e]]).all()
                turn[e] = turn2[e]
    assert episodes >= 1
