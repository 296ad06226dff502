"""TurnBasedManager vs the reference: MultiCorridor, np.random.seed(24),
scripted actions for the agent whose turn it is (fixture recorded from the
reference by tests/golden/make_golden.py multicorridor_turn), and the
reference test's own known answers (tests/test_turn_based_multi_corridor.py)."""
import json
import os

import numpy as np
import pytest

from abmarl_amd.examples import MultiCorridor
from abmarl_amd.managers import TurnBasedManager

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def enc(d):
    return {k: {kk: np.asarray(vv).tolist() for kk, vv in v.items()} for k, v in d.items()}


def test_trajectory_matches_reference():
    recs = json.load(open(os.path.join(GOLDEN, 'multicorridor_turn.json')))
    np.random.seed(24)
    sim = TurnBasedManager(MultiCorridor())
    assert enc(sim.reset()) == recs[0]['reset']
    resets = 0
    for rec in recs[1:]:
        o, r, d, _ = sim.step({k: int(v) for k, v in rec['actions'].items()})
        assert enc(o) == rec['obs']
        assert {k: float(v) for k, v in r.items()} == rec['reward']
        assert {k: bool(v) for k, v in d.items()} == rec['done']
        if 'reset' in rec:
            resets += 1
            assert enc(sim.reset()) == rec['reset']
    assert resets >= 1                          # the cycle carries over a reset


def test_reference_known_answers():
    """tests/test_turn_based_multi_corridor.py:8-60."""
    sim = TurnBasedManager(MultiCorridor())
    assert [next(sim.agent_order) for _ in range(5)] == [f'agent{i}' for i in range(5)]
    np.random.seed(24)
    sim = TurnBasedManager(MultiCorridor())
    obs = sim.reset()
    assert [sim.sim.corridor[i].id for i in range(4, 9)] == \
        ['agent3', 'agent4', 'agent2', 'agent1', 'agent0']
    assert obs == {'agent0': {'left': [True], 'position': [8], 'right': [False]}}
    R = MultiCorridor.Actions.RIGHT
    expect = [('agent1', [True], [7], [False], 0), ('agent2', [True], [6], [False], 0),
              ('agent3', [False], [4], [True], 0), ('agent4', [True], [5], [False], -2)]
    for aid, left, pos, right, rew in expect:
        obs, reward, done, _ = sim.step({k: R for k in obs})
        assert obs == {aid: {'left': left, 'position': pos, 'right': right}}
        assert reward == {aid: rew}
        assert done == {aid: False, '__all__': False}
    obs, reward, done, _ = sim.step({k: R for k in obs})
    assert obs == {'agent0': {'left': [True], 'position': [9], 'right': [False]},
                   'agent1': {'left': [True], 'position': [8], 'right': [False]}}
    assert reward == {'agent0': 100, 'agent1': -1}
    assert done == {'agent0': True, 'agent1': False, '__all__': False}
    with pytest.raises(AssertionError):
        sim.step({'agent0': MultiCorridor.Actions.STAY})
    obs, reward, done, _ = sim.step({'agent1': MultiCorridor.Actions.STAY})
    assert obs == {'agent2': {'left': [True], 'position': [7], 'right': [True]}}
    assert reward == {'agent2': -1}
