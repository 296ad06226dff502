"""The C oracle reproduces the reference's own trajectories bit-exactly
(fixtures generated from /root/reference by tests/golden/make_golden.py)."""
import numpy as np
import pytest

from tests.cases import GOLDEN_CASES, load_golden, golden_config
from tests.golden_replay import replay


class OracleRunner:
    def __init__(self, oracle_mod, g):
        self.cc = golden_config(g)
        c = g['case']
        self.o = oracle_mod.Oracle(self.cc, c['n_envs'])
        self.o.seed(c['seeds'])
        self.obs = self.o.new_obs()
        E, A = self.o.E, self.o.A
        self.rew = np.zeros((E, A), np.float64)
        self.done = np.zeros((E, A), np.uint8)
        self.all_done = np.zeros(E, np.uint8)

    def reset(self, mask):
        err = self.o.reset(self.obs, mask=mask)
        assert not err.any()
        return self.obs.copy()

    def step(self, actions):
        self.o.step(actions, self.obs, self.rew, self.done, self.all_done)
        return self.obs, self.rew, self.done, self.all_done

    def state(self):
        st = self.o.state()
        st['ammo'] = self.o.ammo()
        return st

    def errors(self):
        return self.o.errors()


@pytest.mark.parametrize('name', GOLDEN_CASES)
def test_oracle_matches_reference(oracle_mod, name):
    g = load_golden(name)
    n = replay(OracleRunner(oracle_mod, g), g)
    assert n == g['actions'].shape[0]


def test_shuffle_fixture_needs_the_shuffle(oracle_mod):
    """tb_shuffle (PositionState(randomize_placement_order=True), replayed on
    the GPU through the dict API by test_dict_api.py) is evidence only if the
    shuffled order changes the outcome: placing in agents-dict order from the
    same numpy seeds gives other first observations."""
    import json
    g = load_golden('tb_shuffle')
    c = dict(g['case'])
    c['randomize_placement_order'] = False
    from tests.cases import build_sim
    cc = build_sim(c).compiled()
    o = oracle_mod.Oracle(cc, c['n_envs'])
    o.seed(c['seeds'])
    obs = o.new_obs()
    o.reset(obs)
    assert (obs != g['obs0']).any()
    assert json.loads(json.dumps(g['case']))['randomize_placement_order'] is True


@pytest.mark.parametrize('name', ['tb_shuffle_act', 'rtt_shuffle_act', 'traffic_shuffle_act'])
def test_shuffled_action_fixture_needs_the_shuffle(oracle_mod, name):
    """The *_shuffle_act fixtures (AllStepManager(randomize_action_input=True),
    replayed on the GPU through the dict API by test_dict_api.py) are evidence
    only if the shuffled action order changes the trajectory: the agents-dict
    order from the same seeds and actions diverges from it."""
    g = load_golden(name)
    assert g['case']['randomize_action_input'] is True
    with pytest.raises(AssertionError):
        replay(OracleRunner(oracle_mod, g), g)
