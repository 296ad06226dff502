"""Test-side USER code: a simulation of user components registered beside the
built-in ones (registry.py:58-77).  It is written for this test, not taken
from any example: lantern keepers on a grid hand part of their lamp oil to
the keepers they can see, while blocking wanderers walk around and cut the
lines of sight.

What it exercises in the component plugin API:
  * user state / actor / observer / done classes, registered by type;
  * a user actor that calls create_grid_and_mask (blocking wanderers) on the
    Grid the built-in components maintain;
  * np.random draws in user Python (the initial oil) interleaved with the
    built-in components' draws (PositionState placement, the crowded-cell
    draws of PositionCenteredEncodingObserver) on the one global stream;
  * the built-in PositionState, MoveActor and PositionCenteredEncodingObserver.

`lantern_classes(ns)` builds the classes on a namespace of base classes, so
the SAME user code runs on the reference's components (the fixture
generator, tests/golden/make_comms.py) and on this repository's (the GPU
test, tests/test_registry.py).
"""
import numpy as np


def lantern_classes(ns):
    class Keeper(ns.ObservingAgent, ns.MovingAgent):
        """A lantern keeper: walks, sees `sight` cells far for oil sharing,
        holds `oil` (kept in [0, 2]); `start_oil` None draws it at reset."""

        def __init__(self, sight=None, start_oil=None, **kwargs):
            super().__init__(**kwargs)
            if not (isinstance(sight, int) and sight >= 0):
                raise ValueError('sight: a nonnegative int')
            self.sight = sight
            self.start_oil = start_oil
            self._oil = 0.0

        @property
        def oil(self):
            return self._oil

        @oil.setter
        def oil(self, amount):
            self._oil = 0.0 if amount < 0.0 else (2.0 if amount > 2.0 else float(amount))

    class OilStock(ns.StateBaseComponent):
        """Fills every keeper's lamp (a fixed start or a uniform draw in
        agent order) and keeps a ledger of the oil handed over since each
        keeper last looked."""

        def reset(self, **kwargs):
            self.ledger = {}
            for agent in self.agents.values():
                if isinstance(agent, Keeper):
                    agent.oil = np.random.uniform() if agent.start_oil is None else agent.start_oil
                    self.ledger[agent.id] = 0.0

        def hand_over(self, giver, takers, amount):
            for t in takers:
                t.oil = t.oil + amount
                self.ledger[t.id] += amount
            giver.oil = giver.oil - amount * len(takers)

        def read_and_clear(self, agent):
            got = self.ledger[agent.id]
            self.ledger[agent.id] = 0.0
            return got

    class PourActor(ns.ActorBaseComponent):
        """Action 'pour' in {0, 1, 2}: pour that many tenths of the lamp,
        split evenly between the keepers in sight (the mask of blocking
        wanderers applies) whose encoding `pour_to` lists.  Returns the
        takers, or None when the keeper does not pour."""

        def __init__(self, pour_to=None, oil_stock=None, **kwargs):
            super().__init__(**kwargs)
            self.pour_to = {k: set(v) for k, v in (pour_to or {}).items()}
            self.stock = oil_stock
            for agent in self.agents.values():
                if isinstance(agent, Keeper):
                    agent.action_space[self.key] = ns.Discrete(3)
                    agent.null_action[self.key] = 0

        @property
        def key(self):
            return 'pour'

        @property
        def supported_agent_type(self):
            return Keeper

        def process_action(self, agent, action_dict, **kwargs):
            tenths = int(action_dict.get(self.key, 0)) if isinstance(agent, Keeper) else 0
            if tenths == 0:
                return None
            window, visible = ns.create_grid_and_mask(agent, self.grid, agent.sight, self.agents)
            takers = []
            side = 2 * agent.sight + 1
            for k in range(side * side):
                r, c = divmod(k, side)
                cell = window[r, c]
                if not visible[r, c] or cell is None:
                    continue
                takers.extend(o for o in cell.values() if isinstance(o, Keeper) and o is not agent
                              and o.encoding in self.pour_to.get(agent.encoding, ()))
            if takers:
                self.stock.hand_over(agent, takers, agent.oil * tenths / 10.0 / len(takers))
            return takers

    class OilGauge(ns.ObserverBaseComponent):
        """Observation 'oil': [own oil, oil received since the last look]."""

        def __init__(self, oil_stock=None, **kwargs):
            super().__init__(**kwargs)
            self.stock = oil_stock
            for agent in self.agents.values():
                if isinstance(agent, Keeper):
                    agent.observation_space[self.key] = ns.Box(0, 2, (2,))

        @property
        def key(self):
            return 'oil'

        @property
        def supported_agent_type(self):
            return Keeper

        def get_obs(self, agent, **kwargs):
            if not isinstance(agent, Keeper):
                return {}
            return {self.key: np.array([agent.oil, self.stock.read_and_clear(agent)])}

    class EvenOilDone(ns.DoneBaseComponent):
        """A keeper is done once its oil is within `spread` of the keepers'
        median; all are done when every keeper is."""

        def __init__(self, spread=None, **kwargs):
            super().__init__(**kwargs)
            self.spread = spread

        def _keepers(self):
            return [a for a in self.agents.values() if isinstance(a, Keeper)]

        def get_done(self, agent, **kwargs):
            if not isinstance(agent, Keeper):
                return False
            mid = float(np.median([k.oil for k in self._keepers()]))
            return abs(agent.oil - mid) <= self.spread

        def get_all_done(self, **kwargs):
            return all(self.get_done(k) for k in self._keepers())

    class Wanderer(ns.MovingAgent, ns.GridObservingAgent):
        """Walks around and blocks sight lines."""

        def __init__(self, **kwargs):
            kwargs.setdefault('blocking', True)
            super().__init__(**kwargs)

    class LanternSim(ns.GridWorldSimulation):
        def __init__(self, **kwargs):
            super().__init__(**kwargs)
            self.position_state = ns.PositionState(**kwargs)
            self.oil_stock = OilStock(**kwargs)
            self.move_actor = ns.MoveActor(**kwargs)
            self.pour_actor = PourActor(oil_stock=self.oil_stock, **kwargs)
            self.grid_observer = ns.PositionCenteredEncodingObserver(**kwargs)
            self.oil_gauge = OilGauge(oil_stock=self.oil_stock, **kwargs)
            self.even_done = EvenOilDone(**kwargs)
            self.finalize()

        def reset(self, **kwargs):
            self.position_state.reset(**kwargs)
            self.oil_stock.reset(**kwargs)
            self.rewards = {aid: 0.0 for aid in self.agents}

        def step(self, action_dict, **kwargs):
            # everyone moves first (a failed move costs 0.2), then pours;
            # a pour that reached nobody costs 0.05
            for aid, act in action_dict.items():
                if 'move' in act and not self.move_actor.process_action(self.agents[aid], act, **kwargs):
                    self.rewards[aid] -= 0.2
            for aid, act in action_dict.items():
                takers = self.pour_actor.process_action(self.agents[aid], act, **kwargs)
                if takers is not None and len(takers) == 0:
                    self.rewards[aid] -= 0.05

        def get_obs(self, agent_id, **kwargs):
            agent = self.agents[agent_id]
            obs = dict(self.grid_observer.get_obs(agent, **kwargs))
            obs.update(self.oil_gauge.get_obs(agent, **kwargs))
            return obs

        def get_reward(self, agent_id, **kwargs):
            r = self.rewards[agent_id]
            self.rewards[agent_id] = 0.0
            return r

        def get_done(self, agent_id, **kwargs):
            return self.even_done.get_done(self.agents[agent_id], **kwargs)

        def get_all_done(self, **kwargs):
            return self.even_done.get_all_done(**kwargs)

        def get_info(self, agent_id, **kwargs):
            return {}

    return dict(Keeper=Keeper, OilStock=OilStock, PourActor=PourActor, OilGauge=OilGauge,
                EvenOilDone=EvenOilDone, Wanderer=Wanderer, LanternSim=LanternSim)


USER_COMPONENTS = ('OilStock', 'PourActor', 'OilGauge', 'EvenOilDone')

CASE = dict(rows=6, cols=6, keepers=[(1, 3, None), (1, 4, 0.5), (2, 2, None), (1, 6, None), (1, 2, None)],
            wanderers=[(1, 3), (2, 4), (1, 2)], pour_to={1: [1, 2], 2: [1]}, spread=0.02,
            seeds=[5, 19, 41], n_steps=24, action_seed=303)


def build(classes, c=CASE):
    """keepers: (encoding, sight, start_oil), move range 1; wanderers:
    (move_range, view_range)."""
    agents = {}
    for i, (enc, sight, oil) in enumerate(c['keepers']):
        agents[f'keeper{i}'] = classes['Keeper'](id=f'keeper{i}', encoding=enc, sight=sight, start_oil=oil,
                                                 move_range=1)
    for i, (mr, vr) in enumerate(c['wanderers']):
        agents[f'wanderer{i}'] = classes['Wanderer'](id=f'wanderer{i}', encoding=3, move_range=mr,
                                                     view_range=vr)
    return classes['LanternSim'].build_sim(
        c['rows'], c['cols'], agents=agents, overlapping={1: {1}},
        pour_to={int(k): v for k, v in c['pour_to'].items()}, spread=c['spread'])


def actions(sim, rng, done_agents):
    out = {}
    for aid, a in sim.agents.items():
        if aid in done_agents:
            continue
        out[aid] = {'move': rng.randint(-a.move_range, a.move_range + 1, size=2)}
        if aid.startswith('keeper'):
            out[aid]['pour'] = int(rng.randint(0, 3))
    return out
