"""HIP engine vs the reference's own trajectories (golden fixtures), bit-exact:
observations, float64 reward bits, dones, __all__, positions, health,
active flags and the MT19937 position + key digest after every step."""
import numpy as np
import pytest

from tests.cases import GOLDEN_CASES, load_golden, golden_config
from tests.golden_replay import replay

pytestmark = pytest.mark.gpu


class EngineRunner:
    def __init__(self, g):
        import torch
        from abmarl_amd.engine import GridWorldEngine
        self.torch = torch
        c = g['case']
        self.eng = GridWorldEngine(golden_config(g), c['n_envs'], seeds=c['seeds'])

    def reset(self, mask):
        t = self.torch
        m = None if mask is None else t.as_tensor(mask, device=self.eng.device)
        obs = self.eng.reset(mask=m)
        t.cuda.synchronize()
        assert not self.eng.err.any().item()
        return obs.cpu().numpy()

    def step(self, actions):
        a = self.torch.as_tensor(actions, device=self.eng.device).contiguous()
        obs, rew, done, all_done = self.eng.step(a)
        return obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(), all_done.cpu().numpy()

    def state(self):
        st = self.eng.get_state()
        out = {k: v.cpu().numpy() for k, v in st.items()}
        out['mt'] = out['mt'].view(np.uint32)
        return out


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
    run = EngineRunner(g)
    eng = run.eng
    obs0 = run.reset(None)
    assert (obs0 == g['obs0']).all()
    c = g['case']
    for t in range(g['actions'].shape[0]):
        a = torch.as_tensor(g['actions'][t].astype(np.int32), device=eng.device).contiguous()
        obs, rew, done, ad = eng.step_autoreset(a, horizon=c['horizon'])
        obs, rew, done, ad = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(), ad.cpu().numpy()
        m = g['reset_mask'][t].astype(bool)
        want = np.where(m[:, None, None, None], g['reset_obs'][t], g['obs'][t])
        assert (obs == want).all(), f"step {t}: obs"
        assert (rew.view(np.uint64) == g['reward'][t].view(np.uint64)).all(), f"step {t}: reward"
        assert (done == g['done'][t]).all() and (ad == g['all_done'][t]).all(), f"step {t}: done"
    assert not eng.err.any().item()
