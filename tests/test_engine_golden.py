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


# the workgroup kernel has one view range (rtt_7_views: mixed, the one-wave kernel)
RTT_GOLDEN = [n for n in GOLDEN_CASES if n.startswith('rtt') and n != 'rtt_7_views']


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
