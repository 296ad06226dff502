"""Test-side USER code: a message-broadcasting simulation built from user
components registered beside the built-in ones, in the manner of the
reference's examples/sim/comms_blocking.py (its BroadcastingState /
BroadcastingActor / BroadcastObserver / AverageMessageDone, the ones its
tests/sim/gridworld/test_registry.py:43-55 registers).

The reference's own example cannot be built: BroadcastingAgent derives from
Agent, whose metaclass makes isinstance(x, BroadcastingAgent) true for every
observing-and-acting agent, so the blockers get a 'message' observation
space without a null observation and finalize() asserts.  This version
derives BroadcastingAgent from the observing / acting mixins directly.

`comms_classes(ns)` builds the classes on a namespace of base classes, so
the SAME user code runs on the reference's components (the fixture
generator, tests/golden/make_comms.py) and on this repository's (the GPU
test, tests/test_registry.py).
"""
import numpy as np


def comms_classes(ns):
    class BroadcastingAgent(ns.ObservingAgent, ns.ActingAgent, ns.GridWorldAgent):
        def __init__(self, broadcast_range=None, initial_message=None, **kwargs):
            super().__init__(**kwargs)
            self.broadcast_range = broadcast_range
            self.initial_message = initial_message

        @property
        def broadcast_range(self):
            return self._broadcast_range

        @broadcast_range.setter
        def broadcast_range(self, value):
            assert type(value) is int and value >= 0, "Broadcast Range must be a nonnegative integer."
            self._broadcast_range = value

        @property
        def initial_message(self):
            return self._initial_message

        @initial_message.setter
        def initial_message(self, value):
            if value is not None:
                assert -1 <= value <= 1, "Initial message must be a number between -1 and 1."
            self._initial_message = value

        @property
        def message(self):
            return self._message

        @message.setter
        def message(self, value):
            self._message = min(max(value, -1), 1)

        @property
        def configured(self):
            return super().configured and self.broadcast_range is not None

    class BroadcastingActor(ns.ActorBaseComponent):
        """Broadcast to the visible agents in range whose encoding the
        broadcast mapping names; returns the receivers (None when the agent
        does not broadcast)."""

        def __init__(self, broadcast_mapping=None, **kwargs):
            super().__init__(**kwargs)
            assert type(broadcast_mapping) is dict, "Broadcast mapping must be dictionary."
            self.broadcast_mapping = broadcast_mapping
            for agent in self.agents.values():
                if isinstance(agent, self.supported_agent_type):
                    agent.action_space[self.key] = ns.Discrete(2)

        @property
        def key(self):
            return 'broadcast'

        @property
        def supported_agent_type(self):
            return BroadcastingAgent

        def process_action(self, agent, action_dict, **kwargs):
            if not isinstance(agent, self.supported_agent_type) or not action_dict[self.key]:
                return None
            local, mask = ns.create_grid_and_mask(agent, self.grid, agent.broadcast_range, self.agents)
            out = []
            d = 2 * agent.broadcast_range + 1
            for r in range(d):
                for c in range(d):
                    if mask[r, c] and local[r, c] is not None:
                        for other in local[r, c].values():
                            if other.id != agent.id and \
                                    other.encoding in self.broadcast_mapping[agent.encoding]:
                                out.append(other)
            return out

    class BroadcastingState(ns.StateBaseComponent):
        """Initial messages (np.random.uniform(-1, 1) when unset) and the
        messages each agent received since its last observation."""

        def reset(self, **kwargs):
            for agent in self.agents.values():
                if isinstance(agent, BroadcastingAgent):
                    agent.message = agent.initial_message if agent.initial_message is not None \
                        else np.random.uniform(-1, 1)
            self.receiving_state = {a.id: [] for a in self.agents.values()
                                    if isinstance(a, BroadcastingAgent)}

        def update_receipients(self, from_agent, to_agents):
            for agent in to_agents:
                if agent.id in self.receiving_state:
                    self.receiving_state[agent.id].append((from_agent.id, from_agent.message))

        def update_message_and_reset_receiving(self, agent):
            received, self.receiving_state[agent.id] = self.receiving_state[agent.id], []
            agent.message = np.average([m for _, m in received] + [agent.message])
            return received

    class BroadcastObserver(ns.ObserverBaseComponent):
        def __init__(self, broadcasting_state=None, **kwargs):
            super().__init__(**kwargs)
            self._state = broadcasting_state
            ids = [a.id for a in self.agents.values() if isinstance(a, BroadcastingAgent)]
            for agent in self.agents.values():
                if isinstance(agent, BroadcastingAgent):
                    agent.observation_space[self.key] = ns.Dict({i: ns.Box(-1, 1, (1,)) for i in ids})

        @property
        def key(self):
            return 'message'

        @property
        def supported_agent_type(self):
            return BroadcastingAgent

        def get_obs(self, agent, **kwargs):
            if not isinstance(agent, BroadcastingAgent):
                return {}
            obs = {other: 0 for other in agent.observation_space[self.key]}
            for aid, message in self._state.update_message_and_reset_receiving(agent):
                obs[aid] = message
            obs[agent.id] = agent.message
            return {self.key: obs}

    class AverageMessageDone(ns.DoneBaseComponent):
        def __init__(self, done_tolerance=None, **kwargs):
            super().__init__(**kwargs)
            self.done_tolerance = done_tolerance

        def get_done(self, agent, **kwargs):
            if not isinstance(agent, BroadcastingAgent):
                return False
            avg = np.average([a.message for a in self.agents.values() if isinstance(a, BroadcastingAgent)])
            return bool(np.abs(agent.message - avg) <= self.done_tolerance)

        def get_all_done(self, **kwargs):
            return all(self.get_done(a) for a in self.agents.values() if isinstance(a, BroadcastingAgent))

    class BlockingAgent(ns.MovingAgent, ns.GridObservingAgent):
        def __init__(self, **kwargs):
            super().__init__(blocking=True, **kwargs)

    class BroadcastSim(ns.GridWorldSimulation):
        def __init__(self, **kwargs):
            super().__init__(**kwargs)
            self.position_state = ns.PositionState(**kwargs)
            self.broadcasting_state = BroadcastingState(**kwargs)
            self.move_actor = ns.MoveActor(**kwargs)
            self.broadcast_actor = BroadcastingActor(**kwargs)
            self.grid_observer = ns.PositionCenteredEncodingObserver(**kwargs)
            self.broadcast_observer = BroadcastObserver(broadcasting_state=self.broadcasting_state, **kwargs)
            self.done = AverageMessageDone(**kwargs)
            self.finalize()

        def reset(self, **kwargs):
            self.position_state.reset(**kwargs)
            self.broadcasting_state.reset(**kwargs)
            self.rewards = {agent.id: 0 for agent in self.agents.values()}

        def step(self, action_dict, **kwargs):
            for agent_id, action in action_dict.items():
                agent = self.agents[agent_id]
                receivers = self.broadcast_actor.process_action(agent, action, **kwargs)
                if receivers is not None:
                    self.broadcasting_state.update_receipients(agent, receivers)
            for agent_id, action in action_dict.items():
                agent = self.agents[agent_id]
                if not self.move_actor.process_action(agent, action, **kwargs):
                    self.rewards[agent.id] -= 0.1
            for agent_id in action_dict:
                self.rewards[agent_id] -= 0.01

        def get_obs(self, agent_id, **kwargs):
            agent = self.agents[agent_id]
            return {**self.grid_observer.get_obs(agent, **kwargs),
                    **self.broadcast_observer.get_obs(agent, **kwargs)}

        def get_reward(self, agent_id, **kwargs):
            reward, self.rewards[agent_id] = self.rewards[agent_id], 0
            return reward

        def get_done(self, agent_id, **kwargs):
            return self.done.get_done(self.agents[agent_id], **kwargs)

        def get_all_done(self, **kwargs):
            return self.done.get_all_done(**kwargs)

        def get_info(self, agent_id, **kwargs):
            return {}

    return dict(BroadcastingAgent=BroadcastingAgent, BroadcastingActor=BroadcastingActor,
                BroadcastingState=BroadcastingState, BroadcastObserver=BroadcastObserver,
                AverageMessageDone=AverageMessageDone, BlockingAgent=BlockingAgent,
                BroadcastSim=BroadcastSim)


CASE = dict(rows=7, cols=7, n_broadcasters=4, broadcast_range=6, blockers=[(2, 3), (1, 3), (1, 3)],
            broadcast_mapping={1: [1]}, done_tolerance=5e-10, seeds=[3, 11, 29], n_steps=15,
            action_seed=77)


def build(classes, c=CASE):
    agents = {f'broadcaster{i}': classes['BroadcastingAgent'](
        id=f'broadcaster{i}', encoding=1, broadcast_range=c['broadcast_range'])
        for i in range(c['n_broadcasters'])}
    for i, (mr, vr) in enumerate(c['blockers']):
        agents[f'blocker{i}'] = classes['BlockingAgent'](id=f'blocker{i}', encoding=2, move_range=mr,
                                                         view_range=vr)
    return classes['BroadcastSim'].build_sim(
        c['rows'], c['cols'], agents=agents,
        broadcast_mapping={int(k): v for k, v in c['broadcast_mapping'].items()},
        done_tolerance=c['done_tolerance'])


def actions(sim, rng, done_agents):
    out = {}
    for aid, a in sim.agents.items():
        if aid in done_agents:
            continue
        if hasattr(a, 'broadcast_range'):
            out[aid] = {'broadcast': int(rng.randint(0, 2))}
        else:
            out[aid] = {'move': rng.randint(-a.move_range, a.move_range + 1, size=2)}
    return out
