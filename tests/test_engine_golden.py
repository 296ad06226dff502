"""HIP engine vs the reference's own trajectories (golden fixtures), bit-exact:
observations, float64 reward bits, dones, __all__, positions, health,
active flags and the MT19937 position + key digest after every step."""
import numpy as np
import pytest

from tests.cases import GOLDEN_CASES, load_golden, golden_config
from tests.golden_replay import replay

pytestmark = pytest.mark.gpu


class EngineRunner:
    """The engine behind the fixture's per-ENTITY layout: lane outputs are
    scattered to their entities; static entities (walls) read as the
    reference reports them: obs -2 (not an observer), reward 0, done 1 (not
    an Agent), at their initial position, active, health 0."""

    def __init__(self, g, force_workgroup=False):
        import torch
        from abmarl_amd.engine import GridWorldEngine
        self.torch = torch
        c = g['case']
        self.cc = golden_config(g)
        self.cc.cfg.force_workgroup = int(force_workgroup)
        self.eng = GridWorldEngine(self.cc, c['n_envs'], seeds=c['seeds'])
        self.NE = self.cc.n_agents
        self.lanes = self.eng.lane_entities
        self.E = c['n_envs']

    def _ent(self, x, fill):
        out = np.full((self.E, self.NE) + x.shape[2:], fill, dtype=x.dtype)
        out[:, self.lanes] = x
        return out

    def lane_actions(self, actions):
        return np.ascontiguousarray(actions[:, self.lanes])

    def reset(self, mask):
        t = self.torch
        m = None if mask is None else t.as_tensor(mask, device=self.eng.device)
        self.eng.err.zero_()
        obs = self.eng.reset(mask=m)
        t.cuda.synchronize()
        assert not self.eng.err.any().item()
        return self._ent(obs.cpu().numpy(), -2)

    def step(self, actions):
        a = self.torch.as_tensor(self.lane_actions(actions), device=self.eng.device).contiguous()
        self.eng.err.zero_()
        obs, rew, done, all_done = self.eng.step(a)
        return (self._ent(obs.cpu().numpy(), -2), self._ent(rew.cpu().numpy(), 0.0),
                self._ent(done.cpu().numpy(), 1), all_done.cpu().numpy())

    def state(self):
        st = self.eng.get_state()
        out = {k: v.cpu().numpy() for k, v in st.items()}
        out['mt'] = out['mt'].view(np.uint32)
        pos = np.zeros((self.E, self.NE, 2), np.int32)
        for i, sp in enumerate(self.cc.specs):
            pos[:, i] = (sp.init_row, sp.init_col)
        pos[:, self.lanes] = out['pos']
        out['pos'] = pos
        out['health'] = self._ent(out['health'], 0.0)
        out['flags'] = self._ent(out['flags'], 0x5)    # in grid, active
        out['ammo'] = self._ent(self.eng.get_ammo().cpu().numpy(), 0)
        return out

    def errors(self):
        return self.eng.err.cpu().numpy().astype(np.uint32)


@pytest.mark.parametrize('name', GOLDEN_CASES)
def test_engine_matches_reference(name):
    g = load_golden(name)
    replay(EngineRunner(g), g)


@pytest.mark.parametrize('name', GOLDEN_CASES)
def test_engine_autoreset_matches_reference(name):
    """gw_step_autoreset: terminal reward/done/__all__, and for reset envs the
    next episode's first observation, against the same fixtures."""
    import torch
    g = load_golden(name)
    if 'err' in g and g['err'].any():
        pytest.skip("the reference raised inside a step (covered by the plain replay)")
    run = EngineRunner(g)
    eng = run.eng
    obs0 = run.reset(None)
    assert (obs0 == g['obs0']).all()
    c = g['case']
    for t in range(g['actions'].shape[0]):
        a = torch.as_tensor(run.lane_actions(g['actions'][t].astype(np.int32)),
                            device=eng.device).contiguous()
        obs, rew, done, ad = eng.step_autoreset(a, horizon=c['horizon'])
        obs, rew, done = (run._ent(obs.cpu().numpy(), -2), run._ent(rew.cpu().numpy(), 0.0),
                          run._ent(done.cpu().numpy(), 1))
        ad = ad.cpu().numpy()
        m = g['reset_mask'][t].astype(bool)
        want = np.where(m[:, None, None, None], g['reset_obs'][t], g['obs'][t])
        assert (obs == want).all(), f"step {t}: obs"
        assert (rew.view(np.uint64) == g['reward'][t].view(np.uint64)).all(), f"step {t}: reward"
        assert (done == g['done'][t]).all() and (ad == g['all_done'][t]).all(), f"step {t}: done"
    assert not eng.err.any().item()


# the workgroup kernel has one view range of at most 7 (rtt_7_views: mixed,
# rtt_16_example: ranges 8 and 16 -- the one-wave kernel)
RTT_GOLDEN = [n for n in GOLDEN_CASES if n.startswith('rtt') and n not in ('rtt_7_views', 'rtt_16_example')]


@pytest.mark.parametrize('name', RTT_GOLDEN)
def test_engine_workgroup_kernel_matches_reference(name):
    """The ReachTheTarget workgroup-per-env kernel (gw_rtt.inc) on every RTT
    fixture, the small ones included (gw_config.force_workgroup; config 4's
    size takes it anyway)."""
    g = load_golden(name)
    r = EngineRunner(g, force_workgroup=True)
    assert r.eng.wg
    replay(r, g)


# TeamBattle fixtures with one view range (tb_views mixes them: the one-wave kernel only)
TB_GOLDEN = [n for n in GOLDEN_CASES if n.startswith('tb') and n != 'tb_views']


@pytest.mark.parametrize('name', TB_GOLDEN)
def test_engine_workgroup_team_battle_matches_reference(name):
    """The TeamBattle program on the workgroup-per-env kernel (BinaryAttackActor,
    move isolation, the done components) on every TeamBattle fixture: tb_128
    and tb_100 take it by size (more than 64 lanes), the others are forced."""
    g = load_golden(name)
    r = EngineRunner(g, force_workgroup=True)
    assert r.eng.wg
    replay(r, g)


class ShuffledOrderRunner(EngineRunner):
    """EngineRunner for the *_shuffle_act fixtures (AllStepManager(
    randomize_action_input=True)): before every step, each env's action dict
    -- its live Agents in agents-dict order -- is shuffled with that env's
    Python random stream exactly as all_step_manager.py:62-65 (seeded from
    the fixture's py_seeds before the first reset), and the batch of orders
    goes to the engine (gw_set_action_order)."""

    def __init__(self, g, force_workgroup=False):
        import random
        super().__init__(g, force_workgroup)
        c = g['case']
        self.py = []
        for e in range(self.E):
            random.seed(c['py_seeds'][e])
            self.py.append(random.getstate())
        from abmarl_amd import _abi
        k = np.array([sp.kind for sp in self.cc.specs])
        self.is_agent = ((k & _abi.GW_K_OBSERVING) != 0) & ((k & _abi.GW_K_ACTING) != 0)
        self.lane_of = np.full(self.NE, -1)
        self.lane_of[self.lanes] = np.arange(len(self.lanes))
        self.dead = [set() for _ in range(self.E)]

    def reset(self, mask):
        for e in range(self.E):
            if mask is None or mask[e]:
                self.dead[e] = set()
        return super().reset(mask)

    def step(self, actions):
        import random
        orders = []
        for e in range(self.E):
            live = [i for i in range(self.NE) if self.is_agent[i] and i not in self.dead[e]]
            random.setstate(self.py[e])
            random.shuffle(live)
            self.py[e] = random.getstate()
            first = [int(self.lane_of[i]) for i in live]
            orders.append(first + [k for k in range(len(self.lanes)) if k not in set(first)])
        self.eng.set_action_order(np.array(orders, np.int32))
        obs, rew, done, ad = super().step(actions)
        err = self.errors()
        for e in range(self.E):
            if not (err[e] & 4):
                self.dead[e] |= {i for i in range(self.NE) if self.is_agent[i] and done[e, i]}
        return obs, rew, done, ad


@pytest.mark.parametrize('name,force_workgroup', [
    ('tb_shuffle_act', False), ('rtt_shuffle_act', False), ('rtt_shuffle_act', True),
    ('traffic_shuffle_act', False)])
def test_engine_shuffled_action_order_matches_reference(name, force_workgroup):
    """Batched gw_set_action_order (every env its own shuffled order each
    step) on the one-wave kernel and, for ReachTheTarget, the workgroup-per-env
    kernel, against the reference's own shuffled trajectories."""
    g = load_golden(name)
    r = ShuffledOrderRunner(g, force_workgroup=force_workgroup)
    assert r.eng.wg == force_workgroup
    replay(r, g)
