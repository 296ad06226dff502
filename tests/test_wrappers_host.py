"""Flatten and SuperAgent wrappers on the host, with the reference's own
known answers (tests/test_flatten_wrapper.py, tests/sim/wrappers/
test_super_agent_wrapper.py); the toy simulation below is ours, built to
the behaviour those tests assert (actions recorded, step-count dones)."""
import warnings

import numpy as np
import pytest

from abmarl_amd.spaces import Box, Discrete, MultiBinary, MultiDiscrete, Dict, Tuple
from abmarl_amd.sim.agent_based_simulation import Agent, AgentBasedSimulation
from abmarl_amd.sim.wrappers import (FlattenWrapper, FlattenActionWrapper, SuperAgentWrapper,
                                     BatchedSuperAgents, flatten, unflatten, flatten_space,
                                     flatdim)

box = Box(2, 16, (3, 4), int)
box2 = Box(2.4, 16.1, (3, 4))
discrete = Discrete(11)
multi_binary = MultiBinary(7)
multi_discrete = MultiDiscrete([2, 6, 4])
d = Dict({'first': box2, 'second': multi_binary})
t = Tuple((discrete, box2, multi_discrete))
combo = Tuple((Dict({'first': discrete, 'second': box}), multi_binary))


def test_flatdim():
    """test_flatten_wrapper.py:30-37."""
    assert [flatdim(s) for s in (box, discrete, multi_binary, multi_discrete, d, t, combo)] == \
        [12, 1, 7, 3, 19, 16, 20]


def test_flatten_unflatten_known_answers():
    """test_flatten_wrapper.py:40-135 (values and tolerances as there)."""
    box_s = np.array([[2, 12, 6, 6], [2, 8, 5, 2], [2, 16, 4, 10]])
    np.testing.assert_array_equal(flatten(box, box_s), box_s.reshape(-1))
    np.testing.assert_array_equal(flatten(discrete, 8), [8])
    np.testing.assert_array_equal(flatten(multi_discrete, [0, 3, 1]), [0, 3, 1])
    d_s = {'first': np.arange(12, dtype=float).reshape(3, 4) + 2.5,
           'second': np.array([1, 1, 0, 0, 0, 0, 1])}
    flat_d = flatten(d, d_s)
    assert flat_d.shape == (19,)
    assert np.allclose(flat_d[:12], d_s['first'].reshape(-1), atol=1e-6)
    np.testing.assert_array_equal(flat_d[12:], [1, 1, 0, 0, 0, 0, 1])
    t_s = (6, np.full((3, 4), 3.25), np.array([1, 1, 3]))
    flat_t = flatten(t, t_s)
    assert flat_t[0] == 6 and np.allclose(flat_t[1:13], 3.25) and list(flat_t[13:]) == [1, 1, 3]
    combo_s = ({'first': 2, 'second': np.array([[15, 8, 10, 3], [14, 10, 7, 7], [7, 14, 4, 10]])},
               np.array([1, 1, 1, 0, 1, 1, 0]))
    flat_c = np.array([2, 15, 8, 10, 3, 14, 10, 7, 7, 7, 14, 4, 10, 1, 1, 1, 0, 1, 1, 0])
    np.testing.assert_array_equal(flatten(combo, combo_s), flat_c)
    # unflatten
    assert unflatten(discrete, np.array([8])) == 8
    back = unflatten(d, flat_d)
    assert np.allclose(back['first'], d_s['first'], atol=1e-6)
    np.testing.assert_array_equal(back['second'], d_s['second'])
    bt = unflatten(t, flat_t)
    assert bt[0] == 6 and np.allclose(bt[1], 3.25) and list(bt[2]) == [1, 1, 3]
    bc = unflatten(combo, flat_c)
    assert bc[0]['first'] == 2
    np.testing.assert_array_equal(bc[0]['second'], combo_s[0]['second'])
    np.testing.assert_array_equal(bc[1], combo_s[1])


def test_flatten_space_known_answers():
    """test_flatten_wrapper.py:138-183."""
    assert flatten_space(box) == Box(2, 16, (12,), int)
    assert flatten_space(box2) == Box(2.4, 16.1, (12,))
    assert flatten_space(discrete) == Box(0, 10, (1,), int)
    assert flatten_space(multi_binary) == Box(0, 1, (7,), int)
    assert flatten_space(multi_discrete) == Box(np.array([0, 0, 0]), np.array([1, 5, 3]), (3,), int)
    assert flatten_space(d) == Box(np.array([2.4] * 12 + [0] * 7), np.array([16.1] * 12 + [1] * 7),
                                   (19,))
    assert flatten_space(t) == Box(np.array([0] + [2.4] * 12 + [0, 0, 0]),
                                   np.array([10] + [16.1] * 12 + [1, 5, 3]), (16,))
    fc = flatten_space(combo)
    assert fc == Box(np.array([0] + [2] * 12 + [0] * 7), np.array([10] + [16] * 12 + [1] * 7),
                     (20,), int)
    assert np.issubdtype(fc.dtype, np.integer)
    samp = fc.sample()
    assert all(type(i) is np.int64 for i in samp)
    assert unflatten(combo, samp) in combo


# --------------------------------------------------------------- toy sim
class _Toy(AgentBasedSimulation):
    """Five agents: agent0..agent3 learn, agent4 only observes.  Records the
    last action of each agent; agent i is done once step_count exceeds
    done_at[i]; rewards are fixed per agent."""
    done_at = {'agent0': 3, 'agent1': 35, 'agent2': 8, 'agent3': 30}
    rewards = {'agent0': 2, 'agent1': 3, 'agent2': 5, 'agent3': 7}

    def __init__(self):
        obs = {'agent0': MultiBinary(4), 'agent1': Box(0, 1, (1,), int),
               'agent2': MultiDiscrete([2, 3]),
               'agent3': Dict({'first': Discrete(4), 'second': Box(0, 3, (2,), int)})}
        act = {'agent0': Tuple((Dict({'first': Discrete(3), 'second': Box(-1, 2, (2,))}),
                                MultiBinary(3))),
               'agent1': MultiDiscrete([4, 6, 2]), 'agent2': Dict({'alpha': MultiBinary(3)}),
               'agent3': Tuple((Discrete(3), MultiDiscrete([10, 10]), Discrete(2)))}
        agents = {a: Agent(id=a, observation_space=obs[a], action_space=act[a]) for a in obs}
        from abmarl_amd.sim.agent_based_simulation import ObservingAgent
        agents['agent4'] = ObservingAgent(id='agent4', observation_space=Discrete(2))
        super().__init__(agents=agents)
        self.step_count = 0

    def reset(self, **kw):
        self.action = {a: None for a in self.done_at}
        self.step_count = 0

    def step(self, action, **kw):
        for a, v in action.items():
            self.action[a] = v
        self.step_count += 1

    def get_obs(self, agent_id, **kw):
        return {'agent0': [0, 0, 0, 1], 'agent1': [0], 'agent2': [1, 0],
                'agent3': {'first': 1, 'second': [3, 1]}, 'agent4': 0}[agent_id]

    def get_reward(self, agent_id, **kw):
        return self.rewards[agent_id]

    def get_done(self, agent_id, **kw):
        return self.step_count > self.done_at[agent_id]

    def get_all_done(self, **kw):
        return all(self.get_done(a) for a in self.done_at)

    def get_info(self, agent_id, **kw):
        return self.action[agent_id]


def _super():
    return SuperAgentWrapper(_Toy(), super_agent_mapping={'super0': ['agent0', 'agent3']})


def test_super_agent_mapping_and_spaces():
    sim = _super()
    assert sim._covered_agents == {'agent0', 'agent3'}
    assert sim._uncovered_agents == {'agent1', 'agent2', 'agent4'}
    inner = sim.unwrapped.agents
    assert sim.agents['super0'].action_space == Dict({'agent0': inner['agent0'].action_space,
                                                     'agent3': inner['agent3'].action_space})
    assert sim.agents['super0'].observation_space == Dict({
        'agent0': inner['agent0'].observation_space, 'agent3': inner['agent3'].observation_space,
        'mask': Dict({'agent0': MultiBinary(1), 'agent3': MultiBinary(1)})})
    sim.super_agent_mapping = {'super0': ['agent1', 'agent0'], 'super1': ['agent2', 'agent3']}
    assert sim.agents.keys() == {'super0', 'super1', 'agent4'}
    for bad in (['agent0'], {1: ['agent0']}, {'agent0': ['agent1']}, {'super0': 'agent1'},
                {'super0': [0, 1]}, {'super0': ['agent5']}, {'super0': ['agent4']},
                {'super0': ['agent1', 'agent2'], 'super1': ['agent0', 'agent1']}):
        with pytest.raises(AssertionError):
            SuperAgentWrapper(_Toy(), super_agent_mapping=bad)


def test_super_agent_step_obs_reward_done():
    sim = _super()
    sim.reset()
    a0 = ({'first': 2, 'second': [-1, 2]}, [0, 1, 0])
    a3 = (0, [7, 3], 1)
    sim.step({'super0': {'agent0': a0, 'agent3': a3}, 'agent1': [2, 3, 0],
              'agent2': {'alpha': [1, 1, 1]}})
    assert sim.unwrapped.action == {'agent0': a0, 'agent3': a3, 'agent1': [2, 3, 0],
                                    'agent2': {'alpha': [1, 1, 1]}}
    with pytest.raises(AssertionError):
        sim.step({'agent0': a0})
    assert sim.get_reward('super0') == 9
    # agent0 done: its action is dropped, its obs is reported once, then null
    sim.reset()
    sim.unwrapped.step_count = 4
    sim.step({'super0': {'agent0': a0, 'agent3': a3}})
    assert sim.unwrapped.action['agent0'] is None
    with warnings.catch_warnings(record=True):
        warnings.simplefilter('always')
        first = sim.get_obs('super0')
        assert first == {'agent0': [0, 0, 0, 1], 'agent3': {'first': 1, 'second': [3, 1]},
                         'mask': {'agent0': [False], 'agent3': [True]}}
        sim.unwrapped.agents['agent0'].null_observation = [1, 1, 1, 1]
        assert sim.get_obs('super0')['agent0'] == [1, 1, 1, 1]
    assert sim.get_reward('super0') == 9          # agent0's last reward, once
    assert sim.get_reward('super0') == 7
    sim.unwrapped.step_count = 10
    assert not sim.get_done('super0') and sim.get_done('agent2')
    sim.unwrapped.step_count = 40
    assert sim.get_done('super0') and sim.get_all_done()
    for f in (sim.get_obs, sim.get_reward, sim.get_done):
        with pytest.raises(AssertionError):
            f('agent3')


def test_super_agent_double_wrap():
    sim2 = SuperAgentWrapper(_super(), super_agent_mapping={'double0': ['super0', 'agent1']})
    assert sim2._uncovered_agents == {'agent2', 'agent4'}
    sim2.reset()
    sim2.step({'double0': {'super0': {'agent0': 1, 'agent3': 2}, 'agent1': 3}, 'agent2': 4})
    assert sim2.unwrapped.action == {'agent0': 1, 'agent3': 2, 'agent1': 3, 'agent2': 4}
    assert sim2.get_obs('double0')['mask'] == {'super0': [True], 'agent1': [True]}
    assert sim2.get_reward('double0') == 12
    sim2.unwrapped.step_count = 32
    assert not sim2.get_done('double0')
    sim2.unwrapped.step_count = 40
    assert sim2.get_done('double0')


def test_flatten_wrapper_on_toy():
    sim = FlattenWrapper(_Toy())
    for aid, a in sim.agents.items():
        if isinstance(a, Agent):                  # only learning Agents are flattened
            assert isinstance(a.observation_space, Box) and isinstance(a.action_space, Box)
    assert sim.agents['agent4'].observation_space == Discrete(2)
    sim.reset()
    a0 = ({'first': 2, 'second': [-0.24, 1.9]}, [0, 1, 1])
    sim.step({'agent0': sim.unwrap_action(sim.sim.agents['agent0'], a0)})
    got = sim.get_info('agent0')
    assert got[0]['first'] == 2 and np.allclose(got[0]['second'], [-0.24, 1.9], atol=1e-7)
    np.testing.assert_array_equal(got[1], [0, 1, 1])
    np.testing.assert_array_equal(sim.get_obs('agent3'), [1, 3, 1])
    fa = FlattenActionWrapper(_Toy())
    assert fa.agents['agent3'].observation_space == fa.sim.agents['agent3'].observation_space
    assert fa.agents['agent3'].action_space == Box(np.zeros(4), np.array([2, 9, 9, 1]), (4,), int)


def test_batched_super_agents_host():
    """The batched reduction on lane tensors (CPU tensors; the same ops run on
    the device in the batched env)."""
    import torch

    class _Env:
        agent_ids = ['a0', 'a1', 'a2', 'a3', 'a4']

        class engine:
            device = torch.device('cpu')

    red = BatchedSuperAgents(_Env(), {'s0': ['a0', 'a3'], 's1': ['a1', 'a2', 'a4']})
    reward = torch.tensor([[1.0, 2.0, 4.0, 8.0, 16.0], [0.5, 0, 0, 0.25, 3.0]], dtype=torch.float64)
    done = torch.tensor([[1, 0, 0, 1, 0], [0, 1, 1, 0, 1]], dtype=torch.uint8)
    live = torch.tensor([[0, 1, 1, 0, 1], [1, 0, 0, 1, 0]], dtype=torch.bool)
    r, dn, mask = red.reduce(reward, done, live)
    assert r.tolist() == [[9.0, 22.0], [0.75, 3.0]]
    assert dn.tolist() == [[True, False], [False, True]]
    assert mask.tolist() == [[[False, False, False], [True, True, True]],
                             [[True, True, False], [False, False, False]]]
