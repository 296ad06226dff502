"""AllStepManager control flow vs the reference (BASELINE config 1):
MultiCorridor, np.random.seed(24), scripted actions; fixtures recorded from
the reference by tests/golden/make_golden.py.  Also the reference test's
own known answers (tests/test_all_step_multi_corridor.py:17-60)."""
import json
import os
import random

import numpy as np
import pytest

from abmarl_amd.examples import MultiCorridor
from abmarl_amd.managers import AllStepManager

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def enc(d):
    return {k: {kk: np.asarray(vv).tolist() for kk, vv in v.items()} for k, v in d.items()}


@pytest.mark.parametrize('name,randomize', [('multicorridor', False),
                                            ('multicorridor_shuffled', True)])
def test_trajectory_matches_reference(name, randomize):
    recs = json.load(open(os.path.join(GOLDEN, name + '.json')))
    np.random.seed(24)
    random.seed(24)
    sim = AllStepManager(MultiCorridor(), randomize_action_input=randomize)
    assert enc(sim.reset()) == recs[0]['reset']
    for rec in recs[1:]:
        o, r, d, _ = sim.step({k: int(v) for k, v in rec['actions'].items()})
        assert enc(o) == rec['obs']
        assert {k: float(v) for k, v in r.items()} == rec['reward']
        assert {k: bool(v) for k, v in d.items()} == rec['done']
        if 'reset' in rec:
            assert enc(sim.reset()) == rec['reset']


def test_reference_known_answers():
    np.random.seed(24)
    sim = AllStepManager(MultiCorridor())
    obs = sim.reset()
    assert [sim.sim.corridor[i].id for i in (4, 5, 6, 7, 8)] == \
        ['agent3', 'agent4', 'agent2', 'agent1', 'agent0']
    assert sim.done_agents == set()
    assert obs['agent0'] == {'left': [True], 'position': [8], 'right': [False]}
    assert obs['agent3'] == {'left': [False], 'position': [4], 'right': [True]}
    R = MultiCorridor.Actions.RIGHT
    obs, reward, done, _ = sim.step({f'agent{i}': R for i in range(5)})
    assert obs['agent0'] == {'left': [True], 'position': [9], 'right': [False]}
    assert obs['agent4'] == {'left': [False], 'position': [6], 'right': [True]}
    assert [reward[f'agent{i}'] for i in range(5)] == [100, -1, -1, -5, -3]
    assert done['agent0'] and not done['agent1'] and not done['__all__']
    with pytest.raises(AssertionError):
        sim.step({'agent0': R})
