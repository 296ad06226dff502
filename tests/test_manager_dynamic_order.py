"""DynamicOrderManager and DynamicOrderSimulation.next_agent, restating the
reference's known answers (tests/test_dynamic_order_manager.py:41-102,
tests/sim/test_agent_based_simulation.py:182-215): a four-agent sim whose
actions name the agents that move next; an acting agent is done."""
import pytest

from abmarl_amd.sim import PrincipleAgent, AgentBasedSimulation, DynamicOrderSimulation
from abmarl_amd.managers import DynamicOrderManager


class HandOffSim(DynamicOrderSimulation):
    """Each action is the list of agents whose turn comes next; an agent that
    acted is done."""

    def __init__(self, **kwargs):
        super().__init__(agents={f'agent{i}': PrincipleAgent(id=f'agent{i}') for i in range(4)})

    def reset(self, **kwargs):
        self.finished = set()
        self.next_agent = 'agent3'

    def step(self, action_dict, **kwargs):
        nxt = set()
        for aid, names in action_dict.items():
            self.finished.add(aid)
            nxt.update(names)
        self.next_agent = nxt

    def get_obs(self, agent_id, **kwargs):
        return agent_id

    def get_reward(self, agent_id, **kwargs):
        return {}

    def get_done(self, agent_id, **kwargs):
        return agent_id in self.finished

    def get_all_done(self, **kwargs):
        return all(self.get_done(a) for a in self.agents)

    def get_info(self, agent_id, **kwargs):
        return {}


class PlainSim(AgentBasedSimulation):
    def __init__(self):
        super().__init__(agents={'a': PrincipleAgent(id='a')})

    def reset(self, **kwargs): pass
    def step(self, action, **kwargs): pass
    def get_obs(self, agent_id, **kwargs): return 0
    def get_reward(self, agent_id, **kwargs): return 0
    def get_done(self, agent_id, **kwargs): return False
    def get_all_done(self, **kwargs): return False
    def get_info(self, agent_id, **kwargs): return {}


def test_needs_a_dynamic_order_simulation():
    with pytest.raises(AssertionError):
        DynamicOrderManager(PlainSim())


def test_next_agent_setter():
    # a single id becomes a one-element list; containers are kept as given
    sim = HandOffSim()
    sim.next_agent = 'agent1'
    assert sim.next_agent == ['agent1']
    sim.next_agent = ['agent1', 'agent2']
    assert sim.next_agent == ['agent1', 'agent2']
    sim.next_agent = ('agent3',)
    assert sim.next_agent == ('agent3',)
    sim.next_agent = {'agent0', 'agent1'}
    assert sim.next_agent == {'agent0', 'agent1'}
    with pytest.raises(AssertionError):
        sim.next_agent = 'agent7'
    with pytest.raises(AssertionError):
        sim.next_agent = ['agent0', 'nobody']
    with pytest.raises(AssertionError):
        sim.next_agent = 3


def test_reset_returns_the_first_turn():
    assert DynamicOrderManager(HandOffSim()).reset() == {'agent3': 'agent3'}


def test_stepping_hands_turns_over_and_finishes():
    m = DynamicOrderManager(HandOffSim())
    m.reset()
    obs, _, done, _ = m.step({'agent3': ['agent0', 'agent3']})
    assert obs == {'agent0': 'agent0', 'agent3': 'agent3'}
    assert done == {'agent0': False, 'agent3': True, '__all__': False}
    obs, _, done, _ = m.step({'agent0': ['agent1']})
    assert obs == {'agent1': 'agent1'}
    assert done == {'agent1': False, '__all__': False}
    obs, _, done, _ = m.step({'agent1': ['agent0', 'agent2']})
    assert obs == {'agent0': 'agent0', 'agent2': 'agent2'}
    assert done == {'agent0': True, 'agent2': False, '__all__': False}
    obs, _, done, _ = m.step({'agent2': ['agent1', 'agent2']})
    assert obs == {'agent1': 'agent1', 'agent2': 'agent2'}
    assert done == {'agent1': True, 'agent2': True, '__all__': True}


def test_action_from_an_agent_already_done():
    m = DynamicOrderManager(HandOffSim())
    m.reset()
    m.step({'agent3': ['agent0', 'agent3']})
    with pytest.raises(AssertionError):
        m.step({'agent3': ['agent3'], 'agent0': ['agent1']})


def test_fused_engine_programs_are_refused():
    class Fused(HandOffSim):
        _engine_program = 1
    with pytest.raises(NotImplementedError):
        DynamicOrderManager(Fused())
